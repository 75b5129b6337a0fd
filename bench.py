#!/usr/bin/env python3
"""Benchmark of the nonce-search hot path (BASELINE.json metric: GH/s of the
SHA-256 "msg nonce" min-search at 1/2/4/8 MI355X, and its fraction of the
int32 VALU roofline).

Workloads (--config):
  C2 (default, BASELINE configs[1])  msg "bradfitz", 2^32 nonces per GPU:
      [0, N*2^32-1] over N GPUs (weak scaling; at N = 1 exactly C2's
      [0, 2^32-1]).  The pieces are contiguous; after the warmup they follow
      each GPU's measured rate (the library's range partitioner, DESIGN.md
      §6), so GPUs that clock differently finish together; --no-balance
      keeps rank/device r on [r*2^32, (r+1)*2^32-1].
  C3 (configs[2])  the 120-byte message, 20-digit nonces:
      [2^64 - N*2^32, 2^64-1] (weak scaling).
  C4 (configs[3])  msg "bradfitz", [0, 2^40-1] split over the N GPUs
      (strong scaling; about 20 s per step on one GPU).

How N GPUs are driven (--gpus N):
  * torchrun (WORLD_SIZE = N > 1, the driver's multi-GPU launch): one process
    per GPU.  Each rank opens a rank context of the library on its device
    (LOCAL_RANK, or the one device a per-rank visibility mask leaves it),
    the ranks compare their status, and all of them join one RCCL group
    (rank 0's unique id travels over the rendezvous; the join is bounded).
    Every rank calls bm_search_gpu on the WHOLE range, scans its contiguous
    piece, and one RCCL allgather of 32-byte slots (partial + status) gives
    every rank the answer.  If any rank cannot join, every rank leaves and
    the 16-byte partials of their contexts are gathered over the
    rendezvous; config.parallelism says which combine ran and why.  The
    unique id, the barriers and the max over ranks go through a file
    rendezvous on the node (distributed_bitcoin_minter_amd/rendezvous.py):
    no torch in any rank, so each process maps one HIP runtime, /opt/rocm's,
    the one the GPU test suite runs on, and only the ranks themselves hold
    the GPUs.
  * no launcher, N > 1: ONE process drives N devices (BASELINE C4's design):
    a multi-device context splits the range and combines with
    ncclCommInitAll + ncclAllGather inside the library (host copies if RCCL
    fails at run time, reported in the line).  Fewer than N visible
    devices is an error, unless --rehearse-one-gpu (every "device" is GPU 0,
    partials combined on the host: checks the N-way split, not a measurement).
  * N = 1: one device, no collective.

A step = one complete bm_search_gpu over the workload (every kernel launch,
the second-pass reduction, the combine, the 16-byte result copy); the call is
synchronous, so the step boundary is a device synchronisation.  Timed region:
barrier -> K steps -> barrier, max over ranks.  value = all nonces of all
ranks / that time.  The answer is checked against the committed golden
(tests/golden/) for the workload; a wrong answer exits non-zero.

Also reported:
  roofline      the dominant launch, three ways:
                frac       canonical: algorithmic int32 ops (nonces x C x
                           1384, SURVEY.md §8d, C = SHA-256 blocks the kernel
                           compresses per nonce) / its HIP-event time on the
                           library's stream, vs 78.64 T lane-ops/s per GPU --
                           the metric's own figure, not a ceiling (it can
                           exceed 1 where constant words fold away);
                executed   the VALU lane-ops the kernel really executes per
                           nonce (PMC SQ_INSTS_VALU, else the static count)
                           over the same time, vs 78.64 T and vs the peak at
                           the clock measured under the kernel on this box;
                issue_bound  the ceiling: the kernel loop's issue bound at
                           that clock (measure_clock), and the fraction of
                           it reached;
                plus PMC memory-side bytes from profiles/<round>/.
  rccl_nranks / scaling_valid  (N > 1) what RCCL reported about the
                communicator (ncclCommCount, per rank or device its
                ncclCommUserRank and ncclCommCuDevice, beside each GPU's PCI
                bus id), and whether the line measured N distinct GPUs
                combined the way the run asked for (false, with reasons, on a
                fallback or a one-GPU rehearsal).
  config.ranks / config.devices
                each rank's (device's) nonces, GPU span and rate, and the
                combine that ran.
  cpu_baseline  the oracle's loop shape (format + SHA-256 + strict '<') on this
                host's cores over a bounded sample of C2 (rank 0, N = 1 only);
                "system": one LSP server + N single-threaded CPU miner processes
                + a client over the same window; "optimized": the oracle's
                16-lane AVX-512 scan (a tuned CPU, not the reference's loop) on
                the same cores and window; "go_shape": the loop with
                hash.go's four heap allocations per nonce.
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributed_bitcoin_minter_amd import _lib, codeobj  # noqa: E402
from distributed_bitcoin_minter_amd._lib import (COMBINED_NAMES, Context, device_count,  # noqa: E402
                                                 device_pci_bus_id, rccl_unique_id)
from distributed_bitcoin_minter_amd.dist import calibrated_rates, lex_min, shares_from_rates  # noqa: E402

U64 = (1 << 64) - 1
PER_GPU = 1 << 32
MSG_C2 = b"bradfitz"
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
VALU_PEAK_T = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64 T int32 lane-ops/s (MI355X_MICROARCH.md)
OPS_PER_COMPRESSION = 1384                  # canonical int32 VALU ops
METRIC = "GH/s (SHA-256 \"msg nonce\" min-search) at 1/2/4/8 MI355X; % of int32 VALU peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(config, n):
    """(msg, lower, upper, scaling, description) of a config at n GPUs."""
    if config == "C2":
        return (MSG_C2, 0, n * PER_GPU - 1, "weak",
                "C2: msg 'bradfitz', nonces [0, N*2^32-1], 2^32 per GPU (N > 1: contiguous pieces in proportion to "
                "each GPU's rate measured in the warmup, config.split), inclusive min (hash, nonce)")
    if config == "C3":
        return (M120, U64 - n * PER_GPU + 1, U64, "weak",
                "C3: 120-byte msg, 20-digit nonces [2^64 - N*2^32, 2^64-1], 2^32 per GPU, inclusive min (hash, nonce)")
    if config == "C4":
        return (MSG_C2, 0, (1 << 40) - 1, "strong",
                "C4: msg 'bradfitz', nonces [0, 2^40-1] split over the N GPUs, inclusive min (hash, nonce)")
    raise ValueError(config)


def golden(msg, lo, hi):
    """The committed answer for (msg, [lo, hi]), or None."""
    gdir = os.path.join(ROOT, "tests", "golden")
    cands = []
    for name in ("full_range.json", "scale_ranges.json"):
        try:
            d = json.load(open(os.path.join(gdir, name)))
        except (OSError, ValueError):
            continue
        cands += d.get("cases", []) + [dict(r, msg_hex=d["msg_hex"]) for r in d.get("ranges", [])]
    for c in cands:
        if bytes.fromhex(c["msg_hex"]) == msg and c["lower"] == lo and c["upper"] == hi:
            return [c["hash"], c["nonce"]]
    return None


def compressions_per_nonce(msg_len, digits):
    """Survey C(L, D) = ceil((L+D+10)/64) - floor((L+1)/64):
    whole prefix blocks only counted as midstate."""
    return -(-(msg_len + digits + 10) // 64) - (msg_len + 1) // 64


def kernel_name(p, nbv, pad_block=0):
    """Demangled name of the launch's kernel, as rocprof prints it (without
    the argument list): the folded padding-block layouts are
    search_kernel_padc<P, 1> (pad_block 2: a one-block message) and
    search_kernel_padk<P, K, 1> (pad_block 2 + K: after K prefix blocks),
    search_kernel<P, NBV> otherwise."""
    if pad_block == 2:
        return f"search_kernel_padc<{p}, 1>"
    if pad_block > 2:
        return f"search_kernel_padk<{p}, {pad_block - 2}, 1>"
    return f"search_kernel<{p}, {nbv}>"


def isa_key(p, nbv, pad_block=0):
    """The launch's kernel in isa_mix.json: "P:NBV", "P:c" (padc), "P:kK" (padk)."""
    if pad_block == 2:
        return f"{p}:c"
    if pad_block > 2:
        return f"{p}:k{pad_block - 2}"
    return f"{p}:{nbv}"


def pmc_summary(config, p, nbv=1, pad_block=0):
    """The newest committed rocprofv3 PMC summary entry for the launch's
    kernel under this config (tools/pmc_summary.py: main launches only); PMC
    passes cannot run inside this timed process."""
    pats = [f"pmc_summary_{config}.json"] + (["pmc_summary.json"] if config == "C2" else [])
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")), reverse=True):
        if os.path.basename(path) not in pats:
            continue
        try:
            summ = json.load(open(path))
        except ValueError:
            continue
        for k, e in summ.items():
            if kernel_name(p, nbv, pad_block) in k:
                return e, os.path.relpath(path, ROOT)
    return None, None


def kernel_compressions(L):
    """SHA-256 compressions one launch does per nonce: the varying block,
    plus the constant padding block when the length does not fit (P >= 55);
    an NBV = 2 launch re-compresses the block before once per task of
    10^inner_digits nonces, not once per nonce (tools/len_sweep.py)."""
    return 1 + (1 if L.pad_block else 0) + (L.nbv - 1) / 10 ** L.inner_digits


def issue_bound(key, clock_ghz):
    """gfx950 VALU issue bound of the kernel's inner loop: each
    slow op (v_alignbit, v_add3, SGPR operand, ...) takes an issue slot of its
    own, fast ops of two waves share one, so a SIMD needs max(slow, (slow +
    fast) / 2) slots of 4 cycles per 64 nonces; static counts from
    tools/isa_mix.py on the built assembly, at the clock PMC measured under
    this kernel."""
    path = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "isa_mix.json")
    try:
        lay = json.load(open(path))["layouts"][key]
    except (OSError, KeyError, ValueError):
        return None
    cyc = lay["simd_cycles_per_64_nonces"]
    ghs = 256 * 4 * clock_ghz * 1e9 * 64 / cyc / 1e9
    return {"valu_per_nonce": lay["valu"], "slow": lay["valu_slow"], "fast": lay["valu_fast"],
            "issue_slots_per_nonce": lay["issue_slots"], "clock_ghz": round(clock_ghz, 3),
            "GHs_per_gpu": round(ghs, 2)}


def executed_roofline(nonces, kernel_ms, valu_pmc, pmc_src, valu_static, clock_ghz):
    """The dominant launch against the VALU peak in the instructions it
    really executes: VALU lane-ops per nonce (rocprofv3 SQ_INSTS_VALU x 64 /
    nonces from the committed PMC pass of this config, else the static count
    of the built inner loop, isa_mix.json) x nonces / launch time, as a
    fraction of 78.64 T (2.4 GHz) and of the peak at the clock measured under
    the kernel on this box.  The ceiling for this loop is its issue bound
    (issue_bound.frac); this fraction is below 1 by construction."""
    if valu_pmc:
        v, src = valu_pmc, f"PMC SQ_INSTS_VALU x 64 / nonces (imported: {pmc_src})"
    elif valu_static:
        v, src = valu_static, "static count of the built inner loop (isa_mix.json)"
    else:
        return None
    ach = nonces * v / (kernel_ms * 1e-3) / 1e12
    out = {"valu_per_nonce": v, "src": src, "achieved": round(ach, 3), "unit": "T int32 lane-ops/s",
           "frac": round(ach / VALU_PEAK_T, 4)}
    if clock_ghz:
        peak = VALU_PEAK_T * clock_ghz / 2.4
        out.update(peak_live=round(peak, 2), clock_ghz=round(clock_ghz, 3), frac_live_clock=round(ach / peak, 4))
    return out


class ClockSampler:
    """The driver's gfx clock of one GPU (hwmon freq1_input, found through
    the device's PCI bus id), and its board power where hwmon has it
    (power1_average or power1_input, against power1_cap), sampled every
    `period` s on a host thread, with no change to the kernels.  Silent
    (None) where sysfs does not expose them."""

    def __init__(self, device, period=0.05):
        import threading
        self.period, self.samples, self.watts, self.path, self.ppath, self.cap_w = period, [], [], None, None, None
        if period is None:  # off
            self._thread = None
            return
        try:
            bus = device_pci_bus_id(device).lower()
            hw = sorted(glob.glob(f"/sys/bus/pci/devices/{bus}/hwmon/hwmon*"))
            for h in hw:
                if os.path.exists(os.path.join(h, "freq1_input")):
                    self.path = os.path.join(h, "freq1_input")
                    for name in ("power1_average", "power1_input"):
                        if os.path.exists(os.path.join(h, name)):
                            self.ppath = os.path.join(h, name)
                            break
                    try:
                        with open(os.path.join(h, "power1_cap")) as f:
                            self.cap_w = int(f.read()) / 1e6
                    except (OSError, ValueError):
                        self.cap_w = None
                    break
        except Exception:  # noqa: BLE001 -- informational only
            self.path = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True) if self.path else None

    def _run(self):
        while not self._stop.is_set():
            try:
                with open(self.path) as f:
                    self.samples.append(int(f.read()))
                if self.ppath:
                    with open(self.ppath) as f:
                        self.watts.append(int(f.read()) / 1e6)
            except (OSError, ValueError):
                return
            self._stop.wait(self.period)

    def start(self):
        if self._thread:
            self._thread.start()

    def stop(self):
        """Mean clock in GHz over the samples, or None."""
        if not self._thread:
            return None
        self._stop.set()
        self._thread.join()
        return sum(self.samples) / len(self.samples) / 1e9 if self.samples else None

    def power(self):
        """(mean board power in W, its cap in W), either None where absent."""
        return (sum(self.watts) / len(self.watts) if self.watts else None), self.cap_w


def measure_clock(dev, msg, digits, lo, hi, seconds=0.5, max_nonces=1 << 32):
    """The clock of GPU `dev` while the dominant kernel runs, measured after
    the timed region on a context of its own, over untimed searches of that
    kernel's digit range (at most 2^32 nonces of it), so the step's smaller
    launches (which clock higher) do not bias it:
      * live: the same kernels built with the clock probe
        (libbtcminer_probe.so, `make -C csrc probe`) stamp s_memtime (shader
        cycles) and s_memrealtime (100 MHz) at the start and end of each
        launch: the dominant launch's own average clock;
      * sysfs: the driver's gfx clock (hwmon freq1_input) and board power
        sampled every 10 ms over the same searches.
    Returns {ghz_live, ghz, watts, cap_w, lower, upper, searches} or None."""
    a = max(lo, 10 ** (digits - 1))
    b = min(hi, 10 ** digits - 1, a + max_nonces - 1)
    if a > b:
        return None
    probe = _lib.PROBE_LIB_PATH if os.path.exists(_lib.PROBE_LIB_PATH) else None
    live = []
    with Context(devices=[dev], lib_path=probe) as c:
        c.set_timing(True)
        c.search(msg, a, b)
        smp = ClockSampler(dev, period=0.01)
        smp.start()
        t, k = time.perf_counter(), 0
        while k < 3 or time.perf_counter() - t < seconds:
            c.search(msg, a, b)
            st = c.last_stats()
            dom = max((st.launch[i] for i in range(st.recorded)), key=lambda L: L.nonces, default=None)
            if dom is not None and dom.clock_ghz > 0:
                live.append(dom.clock_ghz)
            k += 1
        ghz = smp.stop()
    watts, cap = smp.power()
    out = {"ghz_live": sum(live) / len(live) if live else None, "ghz": ghz, "watts": watts, "cap_w": cap,
           "lower": a, "upper": b, "searches": k}
    return out if (out["ghz_live"] or ghz) else None


def hip_runtimes():
    """HIP runtime libraries mapped into this process."""
    try:
        maps = open("/proc/self/maps").read().splitlines()
    except OSError:
        return None
    return sorted({ln.split()[-1] for ln in maps if "libamdhip64" in ln})


def cpu_baseline(target_s=3.0):
    """Time the oracle loop (test infrastructure: the CPU 'port' of
    hash.go + miner.go) on this host over a bounded sample of C2: about
    target_s seconds on every core of the box's share (3 s x 16 threads is
    ~48 core-seconds), the system leg over the same window, the optimized
    leg for half as long -- so the GPU is busy for a fair share of the run."""
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
    oracle.search(MSG_C2, hi - n + 1, hi, threads=threads, openssl=True)
    rate = n / (time.perf_counter() - t)
    n = int(min(PER_GPU, max(n, rate * target_s)))
    t = time.perf_counter()
    want = oracle.search(MSG_C2, hi - n + 1, hi, threads=threads, openssl=True)
    dt = time.perf_counter() - t
    out = {"value": n / dt / 1e9, "unit": "GH/s", "cores": threads, "kind": "port",
           "sample": f"msg 'bradfitz', last {n} nonces of [0, 2^32-1] (10-digit, 1 SHA-256 block each), "
                     f"{threads} threads, snprintf-style format + OpenSSL SHA256 + strict '<' per nonce, "
                     f"{dt:.1f} s"}
    try:
        out["system"] = cpu_system_baseline(path, threads, hi - n + 1, hi, want)
    except Exception as e:  # the system leg is informational; the figure above stands alone
        out["system"] = {"error": repr(e)}
    try:
        out["optimized"] = cpu_optimized_baseline(oracle, threads, hi - n + 1, hi, want)
    except Exception as e:  # informational, like the system leg
        out["optimized"] = {"error": repr(e)}
    try:
        out["go_shape"] = cpu_go_shape_baseline(oracle, threads, hi - n + 1, hi, want)
    except Exception as e:  # informational, like the system leg
        out["go_shape"] = {"error": repr(e)}
    return out


def cpu_go_shape_baseline(oracle, threads, lo, hi, want, target_s=1.5):
    """The reference's loop with its per-call allocations (the
    port above formats into one reused buffer, while hash.go:11-15 allocates
    a digest, the Sprintf string, its []byte copy and Sum(nil)'s slice per
    nonce): the same OpenSSL hash, each of those four objects malloc'd and
    freed per nonce, the nonce through printf's %llu (oracle use_openssl = 2).
    Still C, not Go: no garbage collector and no fmt reflection, so it is an
    upper bound on what N Go miner processes reach on these cores."""
    n = 1 << 20
    t = time.perf_counter()
    oracle.search(MSG_C2, hi - n + 1, hi, threads=threads, go_shape=True)
    rate = n / (time.perf_counter() - t)
    n = int(min(hi - lo + 1, max(n, rate * target_s)))
    t = time.perf_counter()
    got = oracle.search(MSG_C2, hi - n + 1, hi, threads=threads, go_shape=True)
    dt = time.perf_counter() - t
    ok = got == want if n == hi - lo + 1 else got == oracle.search(MSG_C2, hi - n + 1, hi, threads=threads,
                                                                   openssl=True)
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": threads, "kind": "port, hash.go allocation shape",
            "seconds": round(dt, 2), "result_ok": ok,
            "sample": f"msg 'bradfitz', last {n} nonces of [0, 2^32-1], {threads} threads, per nonce: malloc'd "
                      f"digest + formatted string (printf %llu) + its copy + 32-byte sum, OpenSSL SHA256, freed"}


def cpu_optimized_baseline(oracle, threads, lo, hi, want, target_s=1.5):
    """Not the reference's loop: the fastest CPU scan this repo has (the
    oracle's 16-lane AVX-512 restatement, oracle/bm_scan16.c: midstate, digits
    stepped in place), on the same window's last nonces, so the GPU is also
    compared with a tuned CPU and not only with the reference's loop shape.
    Its answer must equal the byte-string oracle's over the same nonces."""
    n = 1 << 24
    t = time.perf_counter()
    oracle.search_x16(MSG_C2, hi - n + 1, hi, threads=threads)
    rate = n / (time.perf_counter() - t)
    n = int(min(hi - lo + 1, max(n, rate * target_s)))
    t = time.perf_counter()
    got = oracle.search_x16(MSG_C2, hi - n + 1, hi, threads=threads)
    dt = time.perf_counter() - t
    ok = got == want if n == hi - lo + 1 else got == oracle.search(MSG_C2, hi - n + 1, hi, threads=threads,
                                                                   openssl=True)
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": threads, "kind": "tuned restatement",
            "seconds": round(dt, 2), "result_ok": ok,
            "sample": f"msg 'bradfitz', last {n} nonces of [0, 2^32-1], {threads} threads x 16 AVX-512 lanes, "
                      f"midstate + in-place digit stepping (oracle/bm_scan16.c)"}


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
        got = client.request(hostport, MSG_C2.decode(), hi, p, lower=lo)
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


class Group:
    """Barrier / max / gather across the ranks of this run (one process: trivial)."""

    def __init__(self, rdzv=None):
        self.rdzv = rdzv
        self.rank = rdzv.rank if rdzv else 0
        self.world = rdzv.world if rdzv else 1

    def barrier(self):
        if self.rdzv:
            self.rdzv.barrier()

    def max(self, x):
        return self.rdzv.all_max(x) if self.rdzv else x

    def gather(self, obj):
        return self.rdzv.all_gather(obj) if self.rdzv else [obj]

    def close(self):
        if self.rdzv:
            self.rdzv.close()


def calibrate_split(args, ctx, grp, warm):
    """After the warmup (ranks: at least 2 steps, so at least one is warm):
    each GPU's rate in every warmup step after the first (its own nonces over
    its launches' span, HIP events, so the wait for the other ranks does not
    count; warm: step_record()s), made robust to a transient step
    (dist.calibrated_rates: the median over the steps, a rank held at 0.85 of
    the fastest unless two of its steps agree it is slower) -> integer shares,
    the same on every rank -> the timed steps cut the range in proportion
    (bm_ctx_set_split on every rank's context, joined to the RCCL group or not;
    DESIGN.md §6).  A one-process multi-device context balances itself
    (bm_ctx_set_balance).  Returns what the bench line reports."""
    if args.no_balance or args.warmup < 1:
        return {"mode": "near-equal"}
    if grp.world > 1 and args.warmup < 2:
        # the first call of a process loads each kernel's code object on
        # first launch, which stretches its span: time a warm call
        return {"mode": "near-equal", "note": "the ranks calibrate on the second warmup step"}
    if grp.world == 1:
        if ctx.num_devices() == 1:
            return {"mode": "one device"}
        sh = ctx.get_split()
        return {"mode": "measured device rates (bm_ctx_set_balance)", "shares": sh} if sh else {"mode": "near-equal"}
    mine = [r["nonces"] / r["span_ms"] if r["span_ms"] > 0 and r["nonces"] >= (1 << 30) else 0.0 for r in warm[1:]]
    steps = grp.gather(mine)
    if min(min(r) for r in steps) <= 0:
        return {"mode": "near-equal", "note": "a rank's piece was too small to time"}
    rates, info = calibrated_rates(steps)
    shares = shares_from_rates(rates)
    ctx.set_split(shares)
    return {"mode": f"measured rank rates, median of warmup steps 2..{len(warm)}", "shares": shares,
            "rates_nonces_per_ms": [round(r, 1) for r in rates],
            "step_rates_nonces_per_ms": [[round(x, 1) for x in r] for r in steps],
            "spread": info["spread"], "clamped_to_0.85": info["clamped"]}


def call_roofline(calls, launches, call_nonces, ib=None):
    """roofline.call: the whole call on this device, every launch's
    algorithmic ops (calls: (ops, span_ms) per timed step) over the span of
    its launches.  Two streams overlap launches, which stretches each
    launch's own event time.  With ib (the dominant loop's
    issue bound, one device only), issue_frac = the call's nonces per second
    over that bound: the steadier ceiling figure, since the dominant launch
    shares the GPU with the call's other launches."""
    span = sum(sp for _, sp in calls) / len(calls)
    ach = sum(o for o, _ in calls) / len(calls) / (span * 1e-3) / 1e12
    out = {"achieved": round(ach, 3), "frac": round(ach / VALU_PEAK_T, 4), "span_ms": round(span, 3),
           "launches": launches}
    if ib and ib.get("frac") is not None:
        out["issue_frac"] = round(call_nonces / span / 1e6 / ib["GHs_per_gpu"], 4)
    return out


def _mean(xs):
    return sum(xs) / len(xs) if xs else 0.0


def pci_bus_id(device):
    """The device's PCI bus id (names the physical GPU across processes, whose
    HIP device numbers depend on their visibility masks), or None."""
    try:
        return device_pci_bus_id(device)
    except Exception:  # noqa: BLE001 -- informational
        return None


def step_record(st):
    """What the line keeps of one call's bm_stats_t: nonces, GPU span, the
    combine that ran and RCCL's view of the communicator, per device too, and
    (ABI 7) what the combine and the start cost: the RCCL version, the
    communicator's set-up time, the allgather's event pair (its wait for the
    slowest peer included), the combine's host time, and each device's start
    against the earliest device's."""
    nd = st.devices
    return {"nonces": st.nonces, "span_ms": st.span_ms, "combine": COMBINED_NAMES.get(st.combine_used, "?"),
            "launches": getattr(st, "launches", 0),
            "rccl_status": st.rccl_status, "rccl_nranks": st.rccl_nranks, "rccl_rank": st.rccl_rank,
            "devices": [(st.dev_nonces[i], st.dev_span_ms[i]) for i in range(nd)],
            "dev_rccl": [(st.dev_rccl_rank[i], st.dev_rccl_device[i]) for i in range(nd)],
            "rccl_version": getattr(st, "rccl_version", 0), "rccl_init_ms": getattr(st, "rccl_init_ms", 0.0),
            "allgather_ms": getattr(st, "rccl_allgather_ms", 0.0), "combine_ms": getattr(st, "combine_ms", 0.0),
            "start_threads": getattr(st, "start_threads", 1),
            "dev_start_ms": [getattr(st, "dev_start_ms", [0.0] * nd)[i] for i in range(nd)],
            "dev_allgather_ms": [getattr(st, "dev_allgather_ms", [0.0] * nd)[i] for i in range(nd)]}


def rank_summary(rank, dev, pers, sysfs_clock, start_offset_ms=None):
    """One torchrun rank's share of the timed steps (pers: step() records):
    its GPU (HIP device and PCI bus id), nonces, GPU span and rate, the
    combine that ran, what RCCL reported about the communicator
    (ncclCommCount / ncclCommUserRank / ncclCommCuDevice; 0 / -1 without
    one), its GPU clock over the timed region, what its combine cost per step
    (the allgather's HIP event pair, which includes the wait for the slowest
    rank, and the combine's host time), and when it left the start barrier
    against the earliest rank (wall clock, start_offset_ms)."""
    last = pers[-1]
    mine = {"rank": rank, "device": dev, "pci_bus_id": pci_bus_id(dev), "nonces": last["nonces"],
            "span_ms": round(_mean([p["span_ms"] for p in pers]), 3), "combine": last["combine"],
            "rccl_nranks": last["rccl_nranks"], "rccl_rank": last["rccl_rank"],
            "rccl_device": last["dev_rccl"][0][1] if last["dev_rccl"] else -1,
            "clock_ghz_sysfs": None if sysfs_clock is None else round(sysfs_clock, 3),
            "allgather_ms": round(_mean([p["allgather_ms"] for p in pers]), 4),
            "combine_ms": round(_mean([p["combine_ms"] for p in pers]), 4),
            "rccl_init_ms": round(last["rccl_init_ms"], 1)}
    if start_offset_ms is not None:
        mine["start_offset_ms"] = round(start_offset_ms, 3)
    mine["GHs"] = round(mine["nonces"] / mine["span_ms"] / 1e6, 3) if mine["span_ms"] > 0 else None
    if last["rccl_status"]:
        mine["rccl_status"] = last["rccl_status"]
    return mine


def device_summaries(pers, device_ids):
    """Per device of a one-process context: its HIP device and PCI bus id,
    nonces, span and rate, and its rank in the context's RCCL communicator
    (with the device RCCL placed that rank on)."""
    last = pers[-1]
    slots = []
    for i, (nn, _sp) in enumerate(last["devices"]):
        sp = _mean([p["devices"][i][1] for p in pers])
        r, d = last["dev_rccl"][i] if i < len(last["dev_rccl"]) else (-1, -1)
        slots.append({"device": device_ids[i], "pci_bus_id": pci_bus_id(device_ids[i]), "nonces": nn,
                      "span_ms": round(sp, 3), "GHs": round(nn / sp / 1e6, 3) if sp > 0 else None,
                      "combine": last["combine"], "rccl_nranks": last["rccl_nranks"], "rccl_rank": r,
                      "rccl_device": d,
                      # its first operation against the earliest device's (host
                      # submission; bm_stats_t.dev_start_ms), and its allgather
                      "start_ms": round(_mean([p["dev_start_ms"][i] for p in pers if i < len(p["dev_start_ms"])]),
                                        4),
                      "allgather_ms": round(_mean([p["dev_allgather_ms"][i] for p in pers
                                                   if i < len(p["dev_allgather_ms"])]), 4),
                      # the context's (one communicator set, one combine stage)
                      "rccl_init_ms": round(last["rccl_init_ms"], 1),
                      "combine_ms": round(_mean([p["combine_ms"] for p in pers]), 4)})
    return slots


def rccl_version_str(v):
    """ncclGetVersion's integer (e.g. 22703) as "2.27.3"."""
    if not v:
        return None
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v >= 10000 else f"{v // 1000}.{v // 100 % 10}.{v % 100}"


def rccl_costs(slots, version):
    """N > 1: what the RCCL combine cost per step, from every slot's stats
    (ABI 7): RCCL's version, the communicator's set-up time (the max over
    slots: a rank's init includes its wait for the last rank to arrive), the
    allgather's HIP event pair per step (min and max over slots: every pair
    starts when its own slot's work is done, so it includes the wait for the
    slowest slot, and the min is the closest to the bare collective), and the
    combine stage's host time.  None, with the reason, when no slot combined
    through RCCL (a rendezvous gather, host copies): there is nothing of RCCL
    to report."""
    if not slots or any(s["combine"] != "rccl" for s in slots):
        return {"rccl": None, "rccl_absent": "combine " + "/".join(sorted({s["combine"] for s in slots}))
                + ": no RCCL collective ran"}
    ag = [s.get("allgather_ms", 0.0) for s in slots]
    return {"rccl": {"version": version, "version_str": rccl_version_str(version),
                     "init_ms": round(max(s.get("rccl_init_ms", 0.0) for s in slots), 1),
                     "allgather_ms_min": round(min(ag), 4), "allgather_ms_max": round(max(ag), 4),
                     "combine_ms_max": round(max(s.get("combine_ms", 0.0) for s in slots), 4),
                     "per_step": "allgather_ms: HIP events around each slot's allgather on its stream, from the end "
                                 "of its own work (so the wait for the slowest slot is inside); combine_ms: the "
                                 "library's host time from the end of the slot's own work to the end of its "
                                 "combine (the same wait, the allgather, the result copy)"}}


def warm_layouts(search, msg, lo, hi, per=4096):
    """One tiny untimed search at the start of every digit count of [lo, hi]:
    each layout the range reaches has had its first launch (its code object
    loaded) before a timed step, whatever config the line's own steps ran
    (a C3 line's steps never launch C4's layouts).  Collective
    under a rank group: every rank makes the same calls."""
    calls = 0
    for d in range(len(str(lo)), len(str(hi)) + 1):
        a = max(lo, 10 ** (d - 1) if d > 1 else 0)
        if a > hi:
            break
        search(msg, a, min(hi, a + per - 1))
        calls += 1
    return calls


def c4_block(args, ctx, grp, search, n):
    """north_star's target is stated on a 2^40-nonce search, so
    every line carries one C4 step ([0, 2^40-1], 'bradfitz', strong scaling:
    the N GPUs split it) after the headline's timed region, through the same
    context or group and the same split shares.  Warm: one tiny untimed
    search per digit count first (warm_layouts: P = 9..21, 1- to 13-digit
    nonces).  Timed like the headline (barrier, one search, barrier, max over
    ranks), checked against the committed golden (the 2^40 CPU scan).  About
    20 s on one GPU, 2.5 s on eight."""
    msg, lo, hi, scaling, desc = workload("C4", n)
    warm = warm_layouts(search, msg, lo, hi)
    grp.barrier()
    t_wall = time.time()
    t = time.perf_counter()
    res = search(msg, lo, hi)
    dt = time.perf_counter() - t
    rec = step_record(ctx.last_stats())
    grp.barrier()
    dt = grp.max(dt)
    total = hi - lo + 1
    want = golden(msg, lo, hi)
    out = {"workload": desc, "lower": lo, "upper": hi, "nonces": total, "scaling": scaling,
           "GHs": round(total / dt / 1e9, 4), "seconds": round(dt, 4), "result": list(res), "golden": want,
           "result_ok": None if want is None else list(res) == want, "combine": rec["combine"],
           "warm": f"{warm} untimed searches of {4096} nonces, one per digit count, before the timed one"}
    if grp.world > 1:
        starts = grp.gather(t_wall)
        slots = grp.gather({"rank": grp.rank, "nonces": rec["nonces"], "span_ms": round(rec["span_ms"], 3),
                            "GHs": round(rec["nonces"] / rec["span_ms"] / 1e6, 3) if rec["span_ms"] > 0 else None,
                            "combine": rec["combine"], "allgather_ms": round(rec["allgather_ms"], 4),
                            "start_offset_ms": round((t_wall - min(starts)) * 1e3, 3)})
        out["ranks"] = slots
    else:
        out["devices"] = [{"device": i, "nonces": nn, "span_ms": round(sp, 3),
                           "GHs": round(nn / sp / 1e6, 3) if sp > 0 else None,
                           "start_ms": round(rec["dev_start_ms"][i], 4) if i < len(rec["dev_start_ms"]) else None,
                           "allgather_ms": round(rec["dev_allgather_ms"][i], 4)
                           if i < len(rec["dev_allgather_ms"]) else None}
                          for i, (nn, sp) in enumerate(rec["devices"])]
    return out


# the one-process C4 child: set-up, warm-up and timed steps over N devices
# (N = 2: about 35 s; a one-GPU rehearsal at N = 8: about 25 s); a child that
# hangs costs the line at most this much
ONE_PROCESS_TIMEOUT_S = 180


def c4_one_process(args, grp, n):
    """under torchrun the line measures the rank path, but the Go
    shim (go/bitcoin/miner/gpu.go: bm_ctx_create(0)) and BASELINE configs[3]
    ("one miner process driving 8 x MI355X") are ONE process over N devices:
    bm_ctx_create(N), its per-device submission threads, balance, and
    ncclCommInitAll + one grouped allgather.  So once the line is complete,
    rank 0 measures C4 that way too, in a child process (bench.py --gpus N
    --config C4, no launcher: the one-process mode) under a time limit of its
    own, so that a failure or a hang there cannot cost the line.  Before it
    starts, every rank has closed its context and left the rendezvous, and
    the other ranks have EXITED (rank 0 waits for their pids): idle processes
    that have used a GPU still cost a process beside them on it (on a one-GPU
    rehearsal, 8 idle ranks held the child at 31 of 55 GH/s,
    profiles/r06/rehearse8_c4_one.json).  Called on every rank after
    grp.close(); returns the block on rank 0 and None elsewhere (those ranks
    then exit).  Under a visibility mask that leaves rank 0 fewer than N
    devices the block says why it was skipped; with --rehearse-one-gpu the
    child runs N slots on GPU 0 (host combine; scaling_valid false)."""
    if grp.rank != 0:
        return None
    try:
        return _c4_one_process_child(args, n)
    except Exception as e:  # noqa: BLE001 -- reported in the block, never fatal to the line
        return {"skipped": f"{type(e).__name__}: {e}"[:500]}


def wait_exited(pids, timeout_s=60.0):
    """Until none of `pids` is a live process (the other ranks, after they
    left the rendezvous), or the timeout; returns the pids still alive."""
    def running(pid):
        try:
            os.kill(pid, 0)
        except (ProcessLookupError, PermissionError):  # gone (or a recycled pid that is not ours)
            return False
        try:  # an exited rank its launcher has not reaped yet is a zombie: its GPU is released
            with open(f"/proc/{pid}/stat") as f:
                return f.read().rsplit(")", 1)[1].split()[0] != "Z"
        except (OSError, IndexError):
            return True

    deadline = time.monotonic() + timeout_s
    alive = [pid for pid in pids if running(pid)]  # checked at least once, whatever the timeout
    while alive and time.monotonic() < deadline:
        time.sleep(0.02)
        alive = [pid for pid in alive if running(pid)]
    return alive


def _c4_one_process_child(args, n):
    import subprocess
    have = device_count()
    rehearse = args.rehearse_one_gpu
    if not rehearse and have < n:
        return {"skipped": f"rank 0 sees {have} of {n} devices (a visibility mask): no one-process context "
                           f"over {n} GPUs can open"}
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--gpus", str(n), "--config", "C4", "--no-cpu-baseline",
           "--no-c4", "--clock-seconds", "0", "--steps", "1" if rehearse else "2", "--warmup", "0" if rehearse else "1"]
    if rehearse:
        cmd.append("--rehearse-one-gpu")
    if args.no_balance:
        cmd.append("--no-balance")
    env = child_env(os.environ)  # the child is no torchrun rank: the one-process mode (module docstring)
    t = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=ONE_PROCESS_TIMEOUT_S)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"skipped": f"the one-process child did not finish in {ONE_PROCESS_TIMEOUT_S} s (killed)"}
    wall = time.perf_counter() - t
    lines = [ln for ln in out.strip().splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"skipped": f"the one-process child exited {p.returncode}", "stderr_tail": err[-800:]}
    return one_process_block(json.loads(lines[-1]), n, wall, ["bench.py"] + cmd[3:])


def child_env(environ):
    """The one-process child's environment: the launcher's rank variables
    dropped (it is no torchrun rank), WORLD_SIZE 1; the rest (visibility
    masks, BTCMINER_LIB, ...) kept."""
    env = {k: v for k, v in environ.items()
           if k not in ("RANK", "LOCAL_RANK", "GROUP_RANK", "ROLE_RANK", "LOCAL_WORLD_SIZE", "ROLE_WORLD_SIZE",
                        "GROUP_WORLD_SIZE") and not k.startswith("TORCHELASTIC_")}
    env["WORLD_SIZE"] = "1"
    return env


def one_process_block(line, n, wall, args):
    """The c4_one_process block from the one-process child's bench line."""
    cfg = line["config"]
    blk = {"design": f"one process, {n} devices: bm_ctx_create({n}), a submission thread per device, "
                     "balance, ncclCommInitAll + one grouped allgather (go/bitcoin/miner/gpu.go; BASELINE configs[3])",
           "workload": cfg["workload"], "lower": cfg["lower"], "upper": cfg["upper"], "nonces": cfg["global_nonces"],
           "GHs": line["value"], "seconds": round(line["ms_per_step"] / 1e3, 4), "steps": line["steps"],
           "warmup": line["warmup"], "result": line["result"], "golden": line["golden"],
           "result_ok": line["result_ok"], "parallelism": cfg["parallelism"], "split": cfg["split"],
           "devices": cfg.get("devices"), "rccl_nranks": line.get("rccl_nranks"),
           "scaling_valid": line.get("scaling_valid"), "rccl": line.get("rccl"),
           "start_skew_ms": line.get("start_skew_ms"), "start_threads": line.get("start_threads"),
           "child_wall_s": round(wall, 2), "child_cmd": " ".join(args)}
    for k in ("scaling_invalid", "rccl_absent", "rehearsal"):
        if k in line:
            blk[k] = line[k]
    combines = sorted({d["combine"] for d in cfg.get("devices") or []})
    blk["combine"] = "/".join(combines) if combines else None
    return blk


def scaling_validity(n, slots, want, rehearsal):
    """Whether an N > 1 line measures what it claims: N slots (ranks or
    devices) on N distinct physical GPUs (PCI bus ids), combined the way the
    run asked for -- want = "rccl": every slot combined through one RCCL
    communicator that RCCL itself says has N ranks, numbered 0..N-1; "gather":
    every rank's own partial met over the rendezvous.  A fallback (e.g. a
    group that could not form) or a rehearsal on one GPU makes it false, with
    the reasons listed."""
    why = []
    if rehearsal:
        why.append("rehearsal: every rank / device is GPU 0")
    if len(slots) != n:
        why.append(f"{len(slots)} ranks / devices reported for {n} GPUs")
    buses = [s.get("pci_bus_id") for s in slots]
    if any(b is None for b in buses) or len(set(buses)) != len(buses):
        why.append(f"{len({b for b in buses if b})} distinct GPUs (PCI bus ids) under {len(buses)} ranks / devices")
    combines = sorted({s["combine"] for s in slots})
    if want == "rccl":
        if combines != ["rccl"]:
            why.append(f"combine {'/'.join(combines)} instead of one RCCL allgather")
        else:
            counts = sorted({s["rccl_nranks"] for s in slots})
            if counts != [n]:
                why.append(f"RCCL communicator of {counts} ranks, not {n}")
            if sorted(s["rccl_rank"] for s in slots) != list(range(n)):
                why.append(f"RCCL ranks {sorted(s['rccl_rank'] for s in slots)}, not 0..{n - 1}")
    elif combines != ["local"]:
        why.append(f"combine {'/'.join(combines)} instead of the rendezvous gather of own partials")
    return {"scaling_valid": not why, "scaling_invalid": why} if why else {"scaling_valid": True}


JOIN_TIMEOUT_MS = 120_000  # a group that has not formed by then falls back to the rendezvous gather
PEER_TIMEOUT_MS = 120_000  # a joined rank waits at most this long for the others' partials


def rank_device(args, local):
    """The GPU a torchrun rank drives.  A launcher may give every rank a
    one-device visibility mask (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES per
    rank): then the one visible device is the rank's, whatever its
    LOCAL_RANK.  With several devices visible, LOCAL_RANK picks one."""
    if args.rehearse_one_gpu:
        return 0
    n = device_count()
    if n <= 1:
        return 0  # one device visible (a per-rank mask, or a one-GPU box); none: the context fails loudly
    if local < n:
        return local
    log(f"error: LOCAL_RANK {local} but only {n} HIP devices visible "
        "(--rehearse-one-gpu runs every rank on GPU 0)")
    sys.exit(2)


def open_contexts(args, world, rank, local):
    """(ctx, group, search, parallelism, device) for the launch mode (module
    docstring)."""
    if world > 1:
        from distributed_bitcoin_minter_amd.rendezvous import Rendezvous
        dev = rank_device(args, local)
        grp = Group(Rendezvous())
        # step 1: every rank opens its rank context (its piece of every search,
        # no communicator yet) and the ranks compare notes, so no rank joins
        # RCCL while a peer has already failed
        ctx, err = None, None
        try:
            ctx = Context(devices=[dev], rank=grp.rank, world=grp.world)
        except _lib.BtcMinerError as e:
            err = f"rank {grp.rank}: {e}"
        errs = [x for x in grp.gather(err) if x]
        if errs:
            log(f"error: {errs[0]}")
            if ctx is not None:
                ctx.close()
            grp.close()
            sys.exit(1)
        why = "rehearsal: every rank on GPU 0" if args.rehearse_one_gpu else "--combine gather"
        if args.combine == "rccl" and not args.rehearse_one_gpu:
            # step 2: rank 0's unique id over the rendezvous; every rank joins
            # (non-blocking init, bounded); all or none keep the group
            uid = grp.rdzv.broadcast_bytes(rccl_unique_id() if grp.rank == 0 else None)
            jerr = None
            try:
                ctx.join(uid, timeout_ms=JOIN_TIMEOUT_MS)
            except _lib.BtcMinerError as e:
                jerr = f"rank {grp.rank}: {e}"
            jerrs = [x for x in grp.gather(jerr) if x]
            if not jerrs:
                ctx.set_peer_timeout(PEER_TIMEOUT_MS)
                return ctx, grp, ctx.search, f"{world} processes (one per GPU), RCCL allgather of 32 B slots in-library", dev
            if ctx.joined():
                ctx.leave()
            why = f"RCCL group failed: {jerrs[0]}"
            log(f"rank {grp.rank}: {why}; gathering the partials over the rendezvous instead")

        # each rank's context returns its own piece's partial; the 16-byte
        # partials meet over the rendezvous (the same search; the combine is 16 B)
        def search(msg, lo, hi):
            return lex_min(tuple(p) for p in grp.gather(list(ctx.search(msg, lo, hi))))
        return ctx, grp, search, f"{world} processes (one per GPU), rendezvous gather of 16 B partials ({why})", dev
    grp = Group()
    n = args.gpus
    if n > 1:
        if args.rehearse_one_gpu:
            ctx = Context(devices=[0] * n)  # same device n times: host combine
            return ctx, grp, ctx.search, f"one process, {n}-way split on GPU 0 [rehearsal]", 0
        have = device_count()
        if have < n:
            log(f"error: --gpus {n} but only {have} HIP device(s) visible "
                "(use torchrun for one process per GPU, or --rehearse-one-gpu to check the split on one GPU)")
            sys.exit(2)
        ctx = Context(num_gpus=n)
        return ctx, grp, ctx.search, f"one process, {n} devices", 0
    ctx = Context(devices=[local])
    return ctx, grp, ctx.search, "1 device", local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 40 at C2/C3, about 3 s of GPU time, so a coarse GPU-busy "
                         "sampler sees the card busy; 2 at C4, 20 s each)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 5; 1 at C4)")
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4"])
    ap.add_argument("--combine", default="rccl", choices=["rccl", "gather"],
                    help="torchrun ranks: in-library RCCL allgather (default) or a gather over the rendezvous")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--clock-sample", type=int, default=None,
                    help="1: sample the driver's gfx clock during the timed region (reported, not used); "
                         "default: only at N > 1, where each rank's clock explains the scaling "
                         "(it cost about 0.1%% at N = 1, profiles/r02/s2_sampler_ab.log)")
    ap.add_argument("--clock-seconds", type=float, default=4.0,
                    help="length of the untimed clock measurement after the timed region (measure_clock); "
                         "4 s also keeps the card busy long enough for a coarse GPU-busy sampler to see it, "
                         "whatever --steps the caller passes")
    ap.add_argument("--no-balance", action="store_true",
                    help="keep near-equal pieces (default: after the warmup, pieces follow each GPU's measured rate)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the one warm C4 step ([0, 2^40-1], strong scaling; north_star's target) that every "
                         "C2/C3 line carries after its timed region (about 20 s on one GPU, 2.5 s on eight)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N-way split on ONE GPU (all ranks / devices are GPU 0): exercises the multi-GPU "
                         "path on a one-GPU box; not a scaling measurement")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 2 if args.config == "C4" else 40
    if args.warmup is None:
        args.warmup = 1 if args.config == "C4" else 5

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    _lib.load()  # before anything else can map a second HIP runtime

    ctx, grp, search, how, dev = open_contexts(args, world, rank, local)
    ctx.set_timing(True)
    if world == 1 and ctx.num_devices() > 1 and not args.no_balance:
        ctx.set_balance(True)
    n = args.gpus
    msg, lo, hi, scaling, desc = workload(args.config, n)

    def step():
        res = search(msg, lo, hi)
        st = ctx.last_stats()
        launches = [st.launch[i] for i in range(st.recorded)]
        dom = max(launches, key=lambda L: L.nonces, default=None)
        # this device's algorithmic ops over the call's GPU span (first
        # launch start to last launch end): launches overlap on two streams
        ops = sum(L.nonces * kernel_compressions(L) for L in launches) * OPS_PER_COMPRESSION
        return res, (dom, ops, st.span_ms, step_record(st))

    warm = [step()[1][3] for _ in range(args.warmup)]
    split = calibrate_split(args, ctx, grp, warm)
    sampler = ClockSampler(dev, period=0.05 if (args.clock_sample if args.clock_sample is not None else n > 1)
                           else None)
    grp.barrier()
    t0_wall = time.time()  # when this rank left the barrier (wall clock: common to the node's ranks)
    sampler.start()
    t0 = time.perf_counter()
    doms = []
    res = None
    for _ in range(args.steps):
        res, d = step()
        doms.append(d)
    dt = time.perf_counter() - t0
    sysfs_clock = sampler.stop()
    grp.barrier()
    dt = grp.max(dt)
    clocks = grp.gather(sysfs_clock) if world > 1 else [sysfs_clock]
    starts = grp.gather(t0_wall) if world > 1 else [t0_wall]
    # the clock under the dominant kernel on THIS box, for the issue bound
    # (untimed, after the timed region; every rank on its own GPU)
    dom0 = doms[-1][0]
    box_clock = measure_clock(dev, msg, dom0.digits, lo, hi, seconds=args.clock_seconds) if dom0 is not None else None
    grp.barrier()
    # north_star's 2^40 target, measured at every N: one warm C4
    # step, after the clock measurement so that the issue bound's clock is
    # taken right after the headline's steps, as before
    c4 = None if (args.no_c4 or args.config == "C4") else c4_block(args, ctx, grp, search, n)
    # the same C4 search through ONE process over the N devices
    # (the Go shim's design), measured by rank 0 while the ranks idle

    total = hi - lo + 1
    value = total * args.steps / dt / 1e9
    want = golden(msg, lo, hi)
    dom = doms[-1][0]
    calls = [(o, sp) for _, o, sp, _p in doms if sp > 0]
    pers = [d[3] for d in doms]
    combine = pers[-1]["combine"]
    mean = lambda xs: sum(xs) / len(xs) if xs else 0.0
    if world > 1:
        # each rank's share of the timed steps: its nonces, its GPU span, its
        # rate, how the partials met (and what RCCL says about the
        # communicator), and its GPU clock (driver hwmon)
        slots = grp.gather(rank_summary(grp.rank, dev, pers, sysfs_clock, (t0_wall - min(starts)) * 1e3))
        how += f"; combine {combine}"
    else:
        slots = device_summaries(pers, ([0] * n if args.rehearse_one_gpu else list(range(n))) if n > 1 else [dev])
        if n > 1:
            how += f"; combine {combine}" + (f" (RCCL failed, status {pers[-1]['rccl_status']}: host copies)"
                                             if pers[-1]["rccl_status"] else "")
    out = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "GH/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": desc, "name": args.config, "msg": msg.decode(), "lower": lo, "upper": hi,
                   "global_nonces": total, "parallelism": how, "split": split,
                   ("ranks" if world > 1 else "devices"): slots},
        "result": list(res),
        "golden": want,
        "result_ok": None if want is None else list(res) == want,
        "hip_runtime": hip_runtimes(),
    }
    if c4 is not None:
        out["c4"] = c4
    if n > 1 and world == 1 and c4 is not None:
        # no launcher: this line IS the one-process mode, so its c4 block is
        # the one-process C4 (the field is in every N > 1 line)
        out["c4_one_process"] = {"same_as": "c4", "design": f"one process, {n} devices: this line's own context",
                                 "GHs": c4["GHs"], "seconds": c4["seconds"], "result_ok": c4["result_ok"],
                                 "combine": c4["combine"]}
    if n > 1:
        # what RCCL itself reported (ncclCommCount / UserRank / CuDevice per
        # rank or device) and whether the line measures N distinct GPUs
        # combined the way the run asked for
        out["rccl_nranks"] = (sorted({s["rccl_nranks"] for s in slots}) if world > 1
                              else pers[-1]["rccl_nranks"])
        out.update(scaling_validity(n, slots, args.combine if world > 1 else "rccl", args.rehearse_one_gpu))
        # what RCCL cost per step (ABI 7), or why there is nothing of it
        out.update(rccl_costs(slots, pers[-1]["rccl_version"]))
        # the start of the timed steps: ranks leave the rendezvous barrier at
        # slightly different moments (wall clock); the devices of one process
        # each get their work from a host thread of their own (host submission
        # times, bm_stats_t.dev_start_ms; max over devices, mean over steps)
        if world > 1:
            out["start_skew_ms"] = round((max(starts) - min(starts)) * 1e3, 3)
        else:
            out["start_skew_ms"] = round(_mean([max(p["dev_start_ms"] or [0.0]) for p in pers]), 4)
            out["start_threads"] = pers[-1]["start_threads"]
    if dom is not None:
        ms = [d[0].ms for d in doms if d[0] is not None]
        dom_ms = sum(ms) / len(ms)
        c_eff = kernel_compressions(dom)  # blocks the kernel compresses per nonce
        c_survey = compressions_per_nonce(len(msg), dom.digits)
        achieved = dom.nonces * c_eff * OPS_PER_COMPRESSION / (dom_ms * 1e-3) / 1e12
        key = isa_key(dom.p, dom.nbv, dom.pad_block)  # isa_mix.json key of the kernel
        pmc, pmc_src = pmc_summary(args.config, dom.p, dom.nbv, dom.pad_block)
        pmc = pmc or {}
        cnt = pmc.get("counters", {})
        clock = pmc.get("clock_ghz")
        roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_T, 2),
                "unit": "T int32 lane-ops/s", "frac": round(achieved / VALU_PEAK_T, 4),
                "frac_basis": "canonical: SURVEY.md §8d's 1,384 int32 ops per compression x the blocks the "
                              "kernel compresses per nonce; not a ceiling -- the kernel executes fewer ops per "
                              "nonce than that count (see executed), so this can exceed 1 on layouts whose "
                              "constant words fold away (DESIGN.md §5)",
                # the contract's field; PMC cannot run inside this timed process, so
                # it is the committed pass's figure (roofline.pmc, imported)
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "traffic_unit": "memory-side bytes per launch (PMC FETCH_SIZE+WRITE_SIZE)",
                "traffic_imported": bool(pmc),
                "traffic_note": "imported from roofline.pmc.src (another run); memory-side writes of the dequeue "
                                "counter's returning atomics and of the rare path's spilled best (hash, nonce); "
                                "the search reads no input from HBM (DESIGN.md §5, §8). FETCH_SIZE is not "
                                "doubled: the guide's x2 is for 16-B/lane streaming reads, which this kernel "
                                "does not issue",
                "kernel": f"{kernel_name(dom.p, dom.nbv, dom.pad_block)} ({dom.digits}-digit nonces)",
                "kernel_ms": round(dom_ms, 3), "kernel_nonces": dom.nonces,
                "compressions_per_nonce": c_eff, "ops_per_nonce": c_eff * OPS_PER_COMPRESSION,
                "grid": dom.grid, "tasks_per_thread": dom.tasks_per_thread, "inner_digits": dom.inner_digits}
        if c_survey != c_eff:
            # SURVEY §8d counts only whole prefix blocks as midstate; the planner
            # also folds constant high digits, so the kernel does less work
            roof["survey_compressions_per_nonce"] = c_survey
            roof["survey_frac"] = round(dom.nonces * c_survey * OPS_PER_COMPRESSION / (dom_ms * 1e-3) / 1e12
                                        / VALU_PEAK_T, 4)
        # every PMC-derived figure sits under roofline.pmc, marked
        # as imported from the committed rocprofv3 pass (another run, maybe
        # another box, at that box's clock) -- never measured by this run
        pm = {"src": pmc_src, "imported": True,
              "note": "rocprofv3 --pmc passes cannot run inside this timed process: these figures are the "
                      "committed summary's (tools/pmc_summary.py), not this run's"} if pmc else None
        if pm is not None:
            if pmc.get("valu_per_nonce"):  # SQ_INSTS_VALU x 64 lanes / the profiled launch's nonces
                pm["valu_per_nonce"] = round(pmc["valu_per_nonce"], 1)
            elif "SQ_INSTS_VALU" in cnt and n == 1 and world == 1:
                # an older summary without the profiled launch's nonces: the PMC pass
                # ran this config's N = 1 call, whose dominant launch is this one
                pm["valu_per_nonce"] = round(cnt["SQ_INSTS_VALU"] * 64 / dom.nonces, 1)
            if "SQ_ACTIVE_INST_VALU2" in cnt and cnt.get("SQ_INSTS_VALU"):
                pm["valu_dual_issued_frac"] = round(cnt["SQ_ACTIVE_INST_VALU2"] / cnt["SQ_INSTS_VALU"], 4)
            if clock:
                pm["box_clock_ghz"] = round(clock, 3)
            pm["hbm_bytes_per_launch"] = pmc.get("hbm_bytes_per_launch")
            # is the imported pass about the kernel this run
            # loaded?  Both sides hash the kernel's instruction bytes in the
            # library's gfx950 code object (codeobj.py)
            mine_sha = codeobj.kernel_code_sha(_lib.LIB_PATH, dom.p, dom.nbv, dom.pad_block)
            pm["code_sha"] = pmc.get("code_sha")
            pm["loaded_code_sha"] = mine_sha
            pm["same_kernel"] = (None if not (pmc.get("code_sha") and mine_sha)
                                 else pmc["code_sha"] == mine_sha)
        roof["pmc"] = pm
        # the clock under the dominant kernel on this box: live stamps
        # (s_memtime / s_memrealtime, BM_CLOCK_PROBE builds), else the
        # driver's gfx clock sampled while that kernel's range ran alone
        # (measure_clock).  The committed PMC clock (roofline.pmc) is another
        # run, maybe another box: it is never used for the fraction.
        live = [d[0].clock_ghz for d in doms if d[0] is not None and d[0].clock_ghz > 0]
        live_clock = sum(live) / len(live) if live else None
        if live_clock:
            roof["clock_ghz_live"] = round(live_clock, 3)
        if sysfs_clock:
            # the driver's gfx clock over the whole timed steps (every launch)
            roof["clock_ghz_sysfs"] = round(sysfs_clock, 3)
        box = box_clock or {}
        if box.get("ghz_live"):
            roof["clock_ghz_box_live"] = round(box["ghz_live"], 3)
        if box.get("ghz"):
            roof["clock_ghz_box"] = round(box["ghz"], 3)
        if box.get("watts"):
            # board power while the dominant kernel ran, against its cap: the
            # clock this kernel gets is set by power
            roof["power_w_box"] = round(box["watts"], 1)
            if box.get("cap_w"):
                roof["power_cap_w"] = round(box["cap_w"], 1)
        ib_clock = live_clock or box.get("ghz_live") or box.get("ghz")
        ib = issue_bound(key, ib_clock or clock or 0.0) if (ib_clock or clock) else None
        if ib:
            if ib_clock:
                where = (f"{box.get('searches')} untimed searches of the dominant kernel's range "
                         f"[{box.get('lower')}, {box.get('upper')}] on this box")
                ib["clock_src"] = ("live (s_memtime / s_memrealtime) in the timed launches" if live_clock else
                                   f"live (s_memtime / s_memrealtime, libbtcminer_probe.so) over {where}"
                                   if box.get("ghz_live") else f"hwmon freq1_input every 10 ms over {where}")
                ib["frac"] = round(dom.nonces / (dom_ms * 1e-3) / 1e9 / ib["GHs_per_gpu"], 4)
            else:
                ib["clock_src"] = f"imported: {pmc_src}"
                ib["note"] = "no clock measured on this box: the bound at the committed PMC clock, no frac"
            ib["role"] = "ceiling: the loop's own issue bound at the measured clock (DESIGN.md §5)"
            roof["issue_bound"] = ib
        static = issue_bound(key, 1.0)  # the built loop's static VALU count
        roof["executed"] = executed_roofline(dom.nonces, dom_ms, (pm or {}).get("valu_per_nonce"), pmc_src,
                                             static and static["valu_per_nonce"], ib_clock)
        if calls:
            # the timed steps' own launch count (the context's last call may be
            # the C4 step by now)
            roof["call"] = call_roofline(calls, pers[-1]["launches"], pers[-1]["nonces"],
                                         ib if world == 1 and n == 1 else None)
        out["roofline"] = roof
    if world > 1 and any(c is not None for c in clocks):
        # each rank's GPU clock over the timed region (driver hwmon): what
        # the range partitioner balances against
        out["clock_ghz_sysfs_per_rank"] = [None if c is None else round(c, 3) for c in clocks]
    if args.rehearse_one_gpu:
        out["rehearsal"] = "every rank / device is GPU 0: checks the multi-GPU split and combine, not a measurement"
    if grp.rank == 0 and n == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    ctx.close()
    if world > 1 and c4 is not None:
        # the same C4 search through ONE process over the N
        # devices (the Go shim's design), measured by rank 0 once every other
        # rank has left and exited
        pids = grp.gather(os.getpid())
        grp.close()
        if grp.rank == 0:
            alive = wait_exited(pids[1:])
            blk = c4_one_process(args, grp, n)
            if alive and blk is not None:
                blk["ranks_still_alive"] = alive
            out["c4_one_process"] = blk
    else:
        grp.close()
    if grp.rank == 0:
        print(json.dumps(out), flush=True)
    if out["result_ok"] is False:
        log(f"error: result {out['result']} != golden {want}")
        sys.exit(1)


if __name__ == "__main__":
    main()
