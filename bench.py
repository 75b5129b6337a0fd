#!/usr/bin/env python3
"""Benchmark of the nonce-search hot path (BASELINE.json metric: GH/s of the
SHA-256 "msg nonce" min-search, and its fraction of the int32 VALU roofline).

Workload = BASELINE config C2 (configs[1]): msg "bradfitz", nonces
[0, 2^32-1] on one MI355X, bit-exact min (hash, nonce).  With --gpus N
(torchrun, one process per GPU) the scaling is WEAK: rank r searches
[r*2^32, (r+1)*2^32 - 1] on its own GPU, and the 16-byte partials are
combined with one all_gather over RCCL (the only exchange the path has).

A step = one complete search (all kernel launches, the second-pass
reduction, the 16-byte result copy) of every rank's 2^32 nonces plus the
combine.  value = total nonces of all ranks / max-over-ranks step time.

Also reported:
  roofline      dominant launch (the 10-digit segment) : algorithmic int32
                ops (nonces x C x 1384) / its HIP-event time
                on the library's stream, vs 78.64 T lane-ops/s per GPU.
  cpu_baseline  the CPU oracle's loop shape (format + SHA-256 + strict '<',
                OpenSSL block code) on this host's cores over a bounded
                sample of the same workload (rank 0, N = 1 only); and, under
                "system", the reference's deployment on the same cores: one
                LSP server + N single-threaded CPU miner processes + a client
                over the same window, its answer checked against the oracle.
"""
import argparse
import json
import os
import sys
import time

# torch first: libbtcminer.so then binds to torch's HIP runtime, so the
# process holds exactly one (see tests/conftest.py).
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributed_bitcoin_minter_amd import Context  # noqa: E402
from distributed_bitcoin_minter_amd.dist import combine  # noqa: E402

MSG = b"bradfitz"
PER_GPU = 1 << 32
VALU_PEAK_T = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64 T int32 lane-ops/s (MI355X_MICROARCH.md)
OPS_PER_COMPRESSION = 1384                  # canonical int32 VALU ops


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def compressions_per_nonce(msg_len, digits):
    """C(L, D) = ceil((L+D+10)/64) - floor((L+1)/64)."""
    return -(-(msg_len + digits + 10) // 64) - (msg_len + 1) // 64


def issue_bound(p, nbv=1, clock_ghz=2.37):
    """gfx950 VALU issue bound of the kernel's inner loop: each
    slow op (v_alignbit, v_add3, SGPR operand, ...) takes an issue slot of its
    own, fast ops of two waves share one, so a SIMD needs max(slow, (slow +
    fast) / 2) slots of 4 cycles per 64 nonces; static counts from
    tools/isa_mix.py on the built assembly, clock as measured under this
    kernel (GRBM_GUI_ACTIVE, profiles/r01)."""
    path = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "isa_mix.json")
    try:
        lay = json.load(open(path))["layouts"][f"{p}:{nbv}"]
    except (OSError, KeyError, ValueError):
        return None
    cyc = lay["simd_cycles_per_64_nonces"]
    ghs = 256 * 4 * clock_ghz * 1e9 * 64 / cyc / 1e9
    return {"valu_per_nonce": lay["valu"], "slow": lay["valu_slow"], "fast": lay["valu_fast"],
            "issue_slots_per_nonce": lay["issue_slots"], "clock_ghz": clock_ghz, "GHs_per_gpu": round(ghs, 2)}


def pmc_traffic(p, nbv=1):
    """HBM bytes per launch of search_kernel<p, nbv> from the newest committed
    rocprofv3 PMC summary (FETCH_SIZE + WRITE_SIZE passes, tools/pmc_summary.py);
    PMC passes cannot run inside this timed process."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary.json")), reverse=True):
        try:
            summ = json.load(open(path))
        except ValueError:
            continue
        for k, e in summ.items():
            if f"search_kernel<{p}, {nbv}>" in k and "hbm_bytes_per_launch" in e:
                return e["hbm_bytes_per_launch"], os.path.relpath(path, ROOT), e.get("counters", {})
    return None, None, {}


def cpu_baseline(target_s=10.0):
    """Time the oracle loop (test infrastructure: the CPU 'port' of
    hash.go + miner.go) on this host over a bounded sample of C2."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import Oracle

    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        return None
    oracle = Oracle(path)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    hi = PER_GPU - 1
    n = 1 << 21
    t = time.perf_counter()
    oracle.search(MSG, hi - n + 1, hi, threads=threads, openssl=True)
    rate = n / (time.perf_counter() - t)
    n = int(min(PER_GPU, max(n, rate * target_s)))
    t = time.perf_counter()
    want = oracle.search(MSG, hi - n + 1, hi, threads=threads, openssl=True)
    dt = time.perf_counter() - t
    out = {"value": n / dt / 1e9, "unit": "GH/s", "cores": threads, "kind": "port",
           "sample": f"msg 'bradfitz', last {n} nonces of [0, 2^32-1] (10-digit, 1 SHA-256 block each), "
                     f"{threads} threads, snprintf-style format + OpenSSL SHA256 + strict '<' per nonce, "
                     f"{dt:.1f} s"}
    try:
        out["system"] = cpu_system_baseline(path, threads, hi - n + 1, hi, want)
    except Exception as e:  # the system leg is informational; the figure above stands alone
        out["system"] = {"error": repr(e)}
    return out


# One CPU miner process of the reference's architecture (miner.go:20-74: Join,
# then Request -> sequential strict-'<' scan -> Result), its scan being the
# oracle's single-threaded loop.  Test infrastructure: bench's cpu_baseline leg.
_CPU_MINER = r"""
import sys
root, hostport, lib = sys.argv[1:4]
sys.path[:0] = [root, root + "/tests"]
from conftest import Oracle
from distributed_bitcoin_minter_amd import lsp, miner
from distributed_bitcoin_minter_amd.bitcoin import _as_bytes
o = Oracle(lib)
class Scan:
    def search(self, data, lo, hi):
        return o.search(_as_bytes(data), lo, hi, threads=1, openssl=True)
miner.run(hostport, lsp.Params(EpochLimit=50, EpochMillis=100, WindowSize=1), searcher=Scan())
"""


def cpu_system_baseline(lib, n_miners, lo, hi, want, chunk_bits=24):
    """SURVEY.md §8d CPU baseline as a system: one BitcoinServer + n_miners
    single-threaded CPU miner processes + one client asking for [lo, hi] of
    'bradfitz', all on this host (the reference's deployment: N Go miners
    against one server).  GH/s = nonces / wall time from the request to the
    answer; the answer must equal the oracle's scan of the same window."""
    import subprocess
    import threading
    from distributed_bitcoin_minter_amd import client, lsp
    from distributed_bitcoin_minter_amd.server import BitcoinServer

    p = lsp.Params(EpochLimit=50, EpochMillis=100, WindowSize=1)
    srv = lsp.NewServer(0, p)
    bs = BitcoinServer(srv, chunk=1 << chunk_bits)
    threading.Thread(target=bs.serve, daemon=True).start()
    hostport = f"127.0.0.1:{srv.port}"
    procs = [subprocess.Popen([sys.executable, "-c", _CPU_MINER, ROOT, hostport, lib],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for _ in range(n_miners)]
    try:
        deadline = time.time() + 60
        while bs.stats["joins"] < n_miners:
            if time.time() > deadline or any(q.poll() is not None for q in procs):
                raise RuntimeError(f"only {bs.stats['joins']} of {n_miners} CPU miners joined")
            time.sleep(0.05)
        t = time.perf_counter()
        got = client.request(hostport, MSG.decode(), hi, p, lower=lo)
        dt = time.perf_counter() - t
    finally:
        bs.close()
        for q in procs:
            q.kill()
        for q in procs:
            q.wait()
    n = hi - lo + 1
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": n_miners, "miners": n_miners,
            "chunk": 1 << chunk_bits, "seconds": round(dt, 2), "result_ok": got == want,
            "sample": f"one LSP server + {n_miners} single-threaded CPU miner processes + 1 client on "
                      f"localhost, msg 'bradfitz', nonces [{lo}, {hi}], 2^{chunk_bits}-nonce chunks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 ranks on ONE GPU (every rank uses device 0, gloo combine on CPU): "
                         "exercises the multi-rank path on a one-GPU box; not a scaling measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    cdev = torch.device("cpu") if args.rehearse_one_gpu else dev

    lo = rank * PER_GPU
    hi = lo + PER_GPU - 1
    ctx = Context(devices=[local])
    ctx.set_timing(True)

    def step():
        part = ctx.search(MSG, lo, hi)
        dom = None
        st = ctx.last_stats()
        for i in range(st.recorded):
            L = st.launch[i]
            if dom is None or L.nonces > dom.nonces:
                dom = L
        res = combine(part, device=cdev) if world > 1 else part
        return res, (dom.nonces, dom.ms, dom.digits, dom.p, dom.grid, dom.tasks_per_thread, dom.inner_digits)

    for _ in range(args.warmup):
        res, _ = step()

    def sync():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    sync()
    t0 = time.perf_counter()
    doms = []
    for _ in range(args.steps):
        res, d = step()
        doms.append(d)
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()

    total = PER_GPU * world * args.steps
    value = total / dt / 1e9
    dom_nonces, _, dom_digits, dom_p, dom_grid, dom_tpt, dom_inner = doms[-1]
    dom_ms = sum(d[1] for d in doms) / len(doms)
    C = compressions_per_nonce(len(MSG), dom_digits)
    achieved = dom_nonces * C * OPS_PER_COMPRESSION / (dom_ms * 1e-3) / 1e12
    mix = issue_bound(dom_p)
    traffic, traffic_src, pmc = pmc_traffic(dom_p)
    # measured VALU per nonce (SQ_INSTS_VALU counts wave-instructions: x64 lanes)
    valu_pmc = pmc["SQ_INSTS_VALU"] * 64 / dom_nonces if "SQ_INSTS_VALU" in pmc else None
    # fraction of VALU instructions issued as the second of a same-cycle pair (PMC)
    valu2 = pmc["SQ_ACTIVE_INST_VALU2"] / pmc["SQ_INSTS_VALU"] if "SQ_ACTIVE_INST_VALU2" in pmc else None
    check = None
    if world == 1:
        check = list(res)  # C2 golden: (5256245051, 1626825724)

    out = {
        "metric": "GH/s (SHA-256 \"msg nonce\" min-search) at 1/2/4/8 MI355X; % of int32 VALU peak",
        "value": round(value, 4),
        "unit": "GH/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "C2: msg 'bradfitz', nonces [0, 2^32-1] per GPU (rank r: [r*2^32, (r+1)*2^32-1]), "
                               "inclusive min (hash, nonce)",
                   "msg": MSG.decode(), "nonces_per_gpu": PER_GPU, "global_nonces": PER_GPU * world,
                   "parallelism": f"range-split x{world}" + (", RCCL all_gather of 16 B partials" if world > 1 else "")},
        "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_T, 2),
                     "unit": "T int32 lane-ops/s", "frac": round(achieved / VALU_PEAK_T, 4), "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE+WRITE_SIZE)", "traffic_src": traffic_src,
                     "traffic_note": "the per-launch dequeue counter's returning atomics (64-B memory-side "
                                     "requests); the search reads no input from HBM (DESIGN.md §5)",
                     "valu_per_nonce_pmc": valu_pmc and round(valu_pmc, 1),
                     "valu_dual_issued_frac_pmc": valu2 and round(valu2, 4),
                     "kernel": f"search_kernel<P={dom_p},NBV=1> ({dom_digits}-digit nonces)",
                     "kernel_ms": round(dom_ms, 3), "kernel_nonces": dom_nonces,
                     "ops_per_nonce": C * OPS_PER_COMPRESSION, "grid": dom_grid,
                     "tasks_per_thread": dom_tpt, "inner_digits": dom_inner,
                     "issue_bound": mix and dict(mix, frac=round(dom_nonces / (dom_ms * 1e-3) / 1e9
                                                                  / mix["GHs_per_gpu"], 4))},
        "result": check,
    }
    if args.rehearse_one_gpu:
        out["rehearsal"] = "all ranks on device 0, gloo combine: checks the multi-rank path, not a measurement"
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
