"""bench.py's CPU baseline legs, on CPU (no GPU calls).

cpu_system_baseline is SURVEY.md §8d's baseline as a system: one LSP server,
N single-threaded CPU miner processes (the reference's miner.go:20-74 loop
shape) and one client, all on localhost.  Here it runs at a small size and its
answer must equal the oracle's scan of the same window.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_cpu_system_baseline_small(oracle):
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    lo, hi = 10**10 - 250_000, 10**10 + 250_000 - 1  # across the 10 -> 11 digit boundary
    want = oracle.search(b"bradfitz", lo, hi, threads=4, openssl=True)
    got = bench.cpu_system_baseline(lib, 3, lo, hi, want, chunk_bits=16)
    assert got["result_ok"], got
    assert got["miners"] == 3 and got["value"] > 0


def test_compressions_per_nonce():
    # C1/C2/C4 'bradfitz' one block, C3 (120 B, 20 digits) two
    assert bench.compressions_per_nonce(8, 10) == 1
    assert bench.compressions_per_nonce(8, 13) == 1
    assert bench.compressions_per_nonce(120, 20) == 2
    assert bench.compressions_per_nonce(45, 10) == 2  # 45+10+10 = 65 bytes of padded tail


def test_workloads_and_goldens():
    """Every bench workload at N = 1/2/4/8 has a committed answer where one
    exists: C2 weak ranges [0, N*2^32-1] (scale_ranges.json), C3 at N = 1,
    C4 (the 2^40 CPU scan)."""
    for n in (1, 2, 4, 8):
        msg, lo, hi, scaling, _ = bench.workload("C2", n)
        assert (msg, lo, hi, scaling) == (b"bradfitz", 0, n * 2 ** 32 - 1, "weak")
        assert bench.golden(msg, lo, hi) is not None, n
    msg, lo, hi, _, _ = bench.workload("C3", 1)
    assert hi - lo + 1 == 2 ** 32 and hi == 2 ** 64 - 1 and bench.golden(msg, lo, hi) is not None
    msg, lo, hi, scaling, _ = bench.workload("C4", 8)
    assert (lo, hi, scaling) == (0, 2 ** 40 - 1, "strong")
    assert bench.golden(msg, lo, hi) == [16555811, 890536971553]
    assert bench.golden(b"bradfitz", 0, 12345) is None


def test_multi_gpu_without_devices_fails_loudly():
    """--gpus 2 with no launcher and fewer than 2 visible devices exits 2 with
    a message (never a silent 1-GPU line); a WORLD_SIZE that disagrees with
    --gpus exits 2 too."""
    import subprocess
    from distributed_bitcoin_minter_amd import device_count
    if device_count() >= 2:
        import pytest
        pytest.skip("two or more GPUs visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "--gpus 2" in r.stderr and r.stdout == ""
    env.update(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr


def test_bench_imports_no_torch():
    """The bench process itself never imports torch (torch.distributed runs in
    a file rendezvous), so it maps one HIP runtime."""
    import ast
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    mods = {a.name.split(".")[0] for n in ast.walk(tree) if isinstance(n, ast.Import) for a in n.names}
    mods |= {n.module.split(".")[0] for n in ast.walk(tree) if isinstance(n, ast.ImportFrom) and n.module}
    assert "torch" not in mods


# bench.py's torchrun rank set-up (open_contexts) at world > 1, on CPU: the
# library's Context is replaced by a stand-in whose search is the oracle's
# scan of the rank's piece (a rank context outside a group returns its own
# partial), so the agreement logic over the file rendezvous -- all ranks
# create, all join or all fall back to the rendezvous gather, a failed
# creation stops every rank -- runs for real, with real processes.
_RANK_SETUP = r"""
import json, os, sys, types
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "tests")]
import bench
from conftest import Oracle
from distributed_bitcoin_minter_amd import _lib
from distributed_bitcoin_minter_amd.dist import rank_piece
oracle = Oracle(os.path.join(root, "oracle", "liboracle.so"))
fail = os.environ.get("FAKE_FAIL", "")          # "create:<rank>" or "join:<rank>"
U64 = 2**64 - 1

class FakeCtx:
    def __init__(self, devices=None, rank=None, world=None, **kw):
        self.rank_, self.world_, self.dev, self._joined, self.shares = rank, world, devices[0], False, None
        if fail == f"create:{rank}":
            raise _lib.BtcMinerError(_lib.BM_EHIP, "bm_ctx_create_rank_local")
    def join(self, uid, timeout_ms=0):
        if fail == f"join:{self.rank_}":
            raise _lib.BtcMinerError(_lib.BM_ETIMEDOUT, "bm_ctx_join_rank")
        self._joined = True
    def joined(self): return self._joined
    def leave(self): self._joined = False
    def set_peer_timeout(self, ms): self.timeout = ms
    def set_split(self, s): self.shares = s
    def close(self): pass
    def search(self, msg, lo, hi):
        piece = rank_piece(lo, hi, self.rank_, self.world_, self.shares)
        self.piece = piece
        part = oracle.search(msg, *piece) if piece else (U64, U64)
        if self._joined:   # the in-library allgather: stand in with the whole range
            return oracle.search(msg, lo, hi)
        return part
    def last_stats(self):  # bm_stats_t as the library fills it (ABI 6: RCCL's view of the communicator)
        n = self.piece[1] - self.piece[0] + 1 if self.piece else 0
        j = self._joined
        return types.SimpleNamespace(
            nonces=n, span_ms=1.0, combine_used=_lib.BM_COMBINED_RCCL if j else _lib.BM_COMBINED_LOCAL,
            rccl_status=0, rccl_nranks=self.world_ if j else 0, rccl_rank=self.rank_ if j else -1, devices=1,
            dev_nonces=[n], dev_span_ms=[1.0], dev_rccl_rank=[self.rank_ if j else -1],
            dev_rccl_device=[0 if j else -1],
            # ABI 7: what the library reports of RCCL -- nothing without a group
            rccl_version=22703, rccl_init_ms=40.0 + self.rank_ if j else 0.0,
            rccl_allgather_ms=0.05 + 0.01 * self.rank_ if j else 0.0, combine_ms=0.2 if j else 0.01,
            start_threads=1, dev_start_ms=[0.0], dev_allgather_ms=[0.05 + 0.01 * self.rank_ if j else 0.0])

bench.Context = FakeCtx
bench.device_count = lambda: 1
bench.rccl_unique_id = lambda: os.urandom(128)
# every rank sees one device (a visibility mask), device 0 -- on its own GPU
bench.device_pci_bus_id = lambda d: "0000:%02x:00.0" % (0x10 + int(os.environ.get("FAKE_BUS", os.environ["RANK"])))
args = types.SimpleNamespace(rehearse_one_gpu=False, combine=os.environ.get("COMBINE", "rccl"))
world = int(os.environ["WORLD_SIZE"])
ctx, grp, search, how, dev = bench.open_contexts(args, world, int(os.environ["RANK"]), int(os.environ["LOCAL_RANK"]))
res = search(b"bradfitz", 0, 99_999)
# the line's per-rank summaries and its validity, as main() builds them
rec = bench.step_record(ctx.last_stats())
slots = grp.gather(bench.rank_summary(grp.rank, dev, [rec], None, 0.0))
valid = bench.scaling_validity(world, slots, args.combine, False)
costs = bench.rccl_costs(slots, rec["rccl_version"])
grp.close()
print(json.dumps({"rank": grp.rank, "how": how, "dev": dev, "joined": ctx.joined(), "res": list(res),
                  "slots": slots, "valid": valid, "costs": costs}))
"""


def _rank_setup(world, **env_extra):
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(world), **env_extra)
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK_SETUP, ROOT], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        outs.append((p.returncode, o, e))
    return outs


def test_bench_ranks_join_together(oracle):
    want = list(oracle.search(b"bradfitz", 0, 99_999))
    outs = _rank_setup(3)
    import json
    res = [json.loads(o.strip().splitlines()[-1]) for rc, o, e in outs if rc == 0]
    assert len(res) == 3, [e[-2000:] for _, _, e in outs]
    assert all(r["joined"] and "RCCL allgather" in r["how"] and r["res"] == want for r in res)
    assert all(r["dev"] == 0 for r in res)  # one visible device per rank (a visibility mask): device 0
    # the line shows what RCCL reported -- 3 ranks, numbered 0..2, on 3 distinct GPUs
    for r in res:
        assert [s["rccl_nranks"] for s in r["slots"]] == [3, 3, 3]
        assert [s["rccl_rank"] for s in r["slots"]] == [0, 1, 2]
        assert len({s["pci_bus_id"] for s in r["slots"]}) == 3
        assert r["valid"] == {"scaling_valid": True}, r["valid"]
        # the line's RCCL costs -- version, the slowest init, the
        # allgather's event pair (min / max over ranks), the combine's host time
        c = r["costs"]["rccl"]
        assert (c["version"], c["version_str"], c["init_ms"]) == (22703, "2.27.3", 42.0), c
        assert (c["allgather_ms_min"], c["allgather_ms_max"]) == (0.05, 0.07) and c["combine_ms_max"] == 0.2, c
        assert [s["allgather_ms"] for s in r["slots"]] == [0.05, 0.06, 0.07]


def test_bench_ranks_fall_back_together_when_one_join_fails(oracle):
    """One rank's join fails (here: rank 1 times out): every rank leaves the
    group and the partials meet over the rendezvous; the line says why."""
    import json
    want = list(oracle.search(b"bradfitz", 0, 99_999))
    outs = _rank_setup(3, FAKE_FAIL="join:1")
    res = [json.loads(o.strip().splitlines()[-1]) for rc, o, e in outs if rc == 0]
    assert len(res) == 3, [e[-2000:] for _, _, e in outs]
    for r in res:
        assert not r["joined"] and r["res"] == want
        assert "rendezvous gather" in r["how"] and "RCCL group failed: rank 1" in r["how"], r["how"]
        # --combine rccl that fell back: not a valid scaling line, and it says why
        assert r["valid"]["scaling_valid"] is False
        assert any("instead of one RCCL allgather" in w for w in r["valid"]["scaling_invalid"]), r["valid"]
        assert all(s["rccl_nranks"] == 0 and s["combine"] == "local" for s in r["slots"])
        # the rendezvous path ran no RCCL collective: no RCCL costs, and the reason
        assert r["costs"] == {"rccl": None, "rccl_absent": "combine local: no RCCL collective ran"}, r["costs"]
        assert all(s["allgather_ms"] == 0 and s["rccl_init_ms"] == 0 for s in r["slots"])
    outs = _rank_setup(2, COMBINE="gather")
    res = [json.loads(o.strip().splitlines()[-1]) for rc, o, e in outs if rc == 0]
    assert len(res) == 2 and all("--combine gather" in r["how"] and r["res"] == want for r in res)
    assert all(r["valid"] == {"scaling_valid": True} for r in res)  # the combine the run asked for
    # ranks that share one GPU (same PCI bus id): never a valid scaling line
    outs = _rank_setup(2, COMBINE="gather", FAKE_BUS="0")
    res = [json.loads(o.strip().splitlines()[-1]) for rc, o, e in outs if rc == 0]
    assert len(res) == 2 and all(r["valid"]["scaling_valid"] is False for r in res)
    assert all(any("1 distinct GPUs" in w for w in r["valid"]["scaling_invalid"]) for r in res)


def test_bench_ranks_stop_together_when_one_context_fails():
    """A rank whose context cannot be created stops every rank (exit 1, the
    failing rank named) before any of them joins RCCL: no rank is left
    waiting in a communicator for it."""
    outs = _rank_setup(3, FAKE_FAIL="create:2")
    assert [rc for rc, _, _ in outs] == [1, 1, 1], outs
    assert all("rank 2" in e for _, _, e in outs)


def test_kernel_compressions_per_nonce():
    """The roofline counts the blocks a launch really compresses per nonce:
    1 for the plain layouts, 2 with the constant padding block, and for an
    NBV = 2 launch 1 + 1/task (the block before is re-compressed once per
    task of 10^inner_digits nonces)."""
    from types import SimpleNamespace as L
    assert bench.kernel_compressions(L(nbv=1, pad_block=0, inner_digits=2)) == 1
    assert bench.kernel_compressions(L(nbv=1, pad_block=1, inner_digits=2)) == 2
    assert bench.kernel_compressions(L(nbv=1, pad_block=2, inner_digits=2)) == 2  # search_kernel_padc
    assert bench.kernel_compressions(L(nbv=2, pad_block=0, inner_digits=2)) == 1.01
    assert bench.kernel_compressions(L(nbv=2, pad_block=0, inner_digits=1)) == 1.1


def test_scaling_validity_cases():
    """bench.scaling_validity: an N > 1 line is valid only for N slots on N
    distinct GPUs combined the way the run asked for; RCCL must itself report
    N ranks numbered 0..N-1."""
    def slot(i, bus=None, combine="rccl", nranks=4, rank=None):
        return {"pci_bus_id": bus or f"0000:{i:02x}:00.0", "combine": combine, "rccl_nranks": nranks,
                "rccl_rank": i if rank is None else rank}
    ok = [slot(i) for i in range(4)]
    assert bench.scaling_validity(4, ok, "rccl", False) == {"scaling_valid": True}
    v = bench.scaling_validity(4, ok, "rccl", True)
    assert v["scaling_valid"] is False and "rehearsal" in v["scaling_invalid"][0]
    v = bench.scaling_validity(4, [slot(i, nranks=1, rank=0) for i in range(4)], "rccl", False)
    assert not v["scaling_valid"] and any("of [1] ranks" in w for w in v["scaling_invalid"])
    v = bench.scaling_validity(4, [slot(i, combine="host") for i in range(4)], "rccl", False)
    assert not v["scaling_valid"] and "combine host" in v["scaling_invalid"][0]
    v = bench.scaling_validity(4, ok[:3], "rccl", False)
    assert not v["scaling_valid"]
    v = bench.scaling_validity(2, [slot(0, bus="x", nranks=2), slot(1, bus="x", nranks=2)], "rccl", False)
    assert not v["scaling_valid"] and "1 distinct GPUs" in v["scaling_invalid"][0]
    assert bench.scaling_validity(2, [slot(i, combine="local") for i in range(2)], "gather", False)["scaling_valid"]


def test_executed_roofline():
    """roofline.executed: executed VALU lane-ops (PMC when committed, else the
    static count) over the launch time, against 78.64 T and the live-clock
    peak; C2's round-3 figures give about 0.885."""
    e = bench.executed_roofline(2 ** 32, 2 ** 32 / 55.5e6, 1254.0, "p.json", 1250, 2.25)
    assert e["valu_per_nonce"] == 1254.0 and "PMC" in e["src"]
    assert abs(e["frac"] - 0.885) < 0.002
    assert abs(e["frac_live_clock"] - e["frac"] * 2.4 / 2.25) < 1e-3
    e = bench.executed_roofline(10 ** 9, 20.0, None, None, 1250, None)
    assert e["valu_per_nonce"] == 1250 and "static" in e["src"] and "frac_live_clock" not in e
    assert bench.executed_roofline(1, 1.0, None, None, None, 2.0) is None


def test_call_roofline():
    """roofline.call: the call's ops over its launches' span, and (one device)
    its nonces per second against the dominant loop's issue bound; the
    round-4 check run (profiles/r04/call_issue_frac.log) gives 0.971."""
    ops = (2 ** 32) * bench.OPS_PER_COMPRESSION
    c = bench.call_roofline([(ops, 80.6), (ops, 80.616)], 11, 2 ** 32, {"frac": 0.97, "GHs_per_gpu": 54.86})
    assert c["launches"] == 11 and c["span_ms"] == 80.608
    assert abs(c["achieved"] - 73.74) < 0.01 and abs(c["frac"] - c["achieved"] / bench.VALU_PEAK_T) < 1e-4
    assert c["issue_frac"] == 0.9712
    assert "issue_frac" not in bench.call_roofline([(ops, 80.6)], 11, 2 ** 32, None)
    assert "issue_frac" not in bench.call_roofline([(ops, 80.6)], 11, 2 ** 32, {"GHs_per_gpu": 54.86, "frac": None})


def test_one_process_device_summaries(monkeypatch):
    """The one-process N-device line: each device slot carries its HIP device,
    PCI bus id and its rank in the context's RCCL communicator (from the
    stats' dev_rccl_*), and scaling_validity reads them: RCCL over 4 distinct
    devices is valid; the host-copy fallback (no ranks) is not."""
    from types import SimpleNamespace as NS
    monkeypatch.setattr(bench, "device_pci_bus_id", lambda d: f"0000:{0x20 + d:02x}:00.0")

    def stats(combine, nranks):
        return NS(nonces=4 << 30, span_ms=80.0, combine_used=combine, rccl_status=0 if nranks else -4,
                  rccl_nranks=nranks, rccl_rank=0 if nranks else -1, devices=4, dev_nonces=[1 << 30] * 4,
                  dev_span_ms=[79.0, 80.0, 78.5, 79.5], dev_rccl_rank=list(range(4)) if nranks else [-1] * 4,
                  dev_rccl_device=list(range(4)) if nranks else [-1] * 4)
    from distributed_bitcoin_minter_amd import _lib
    slots = bench.device_summaries([bench.step_record(stats(_lib.BM_COMBINED_RCCL, 4))], [0, 1, 2, 3])
    assert [s["rccl_rank"] for s in slots] == [0, 1, 2, 3] and [s["rccl_device"] for s in slots] == [0, 1, 2, 3]
    assert len({s["pci_bus_id"] for s in slots}) == 4 and all(s["combine"] == "rccl" for s in slots)
    assert bench.scaling_validity(4, slots, "rccl", False) == {"scaling_valid": True}
    # ABI 7 figures absent from this stand-in: zeros, and the RCCL block still forms
    assert [s["start_ms"] for s in slots] == [0.0] * 4 and bench.rccl_costs(slots, 0)["rccl"]["version_str"] is None
    slots = bench.device_summaries([bench.step_record(stats(_lib.BM_COMBINED_HOST, 0))], [0, 1, 2, 3])
    v = bench.scaling_validity(4, slots, "rccl", False)
    assert v["scaling_valid"] is False and "combine host" in v["scaling_invalid"][0]


def test_kernel_names_and_isa_keys():
    """The launch stats' pad_block names the kernel rocprof prints and its
    isa_mix.json entry: 2 = search_kernel_padc<P, 1>, 2 + K =
    search_kernel_padk<P, K, 1>, and every padk layout has a
    static count there with no more issue slots than the generic kernel's."""
    import json
    assert bench.kernel_name(18, 1) == "search_kernel<18, 1>" and bench.isa_key(18, 1) == "18:1"
    assert bench.kernel_name(60, 1, 2) == "search_kernel_padc<60, 1>" and bench.isa_key(60, 1, 2) == "60:c"
    assert bench.kernel_name(60, 1, 4) == "search_kernel_padk<60, 2, 1>" and bench.isa_key(60, 1, 4) == "60:k2"
    lay = json.load(open(os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc", "isa_mix.json")))["layouts"]
    for p in range(55, 64):
        for k in range(1, 16):  # round 6: K = 3..15 too (messages up to 1,024 bytes)
            assert lay[f"{p}:k{k}"]["issue_slots"] <= lay[f"{p}:1"]["issue_slots"], (p, k)
            assert lay[f"{p}:k{k}"]["readlanes"] == 0, (p, k)  # no spilled SGPR read back per nonce
    assert lay["56:1"]["readlanes"] == 24  # the generic kernel's (messages with >= 16 prefix blocks)
    # round 6: the NBV = 2 inner loops read no spilled SGPR back (isa_mix's old
    # pick, the per-task block, showed 21 and 17 for these two)
    assert lay["13:2"]["readlanes"] == 0 and lay["14:2"]["readlanes"] == 0
    assert bench.kernel_name(60, 1, 17) == "search_kernel_padk<60, 15, 1>" and bench.isa_key(60, 1, 17) == "60:k15"
    assert bench.issue_bound("60:k1", 2.4)["GHs_per_gpu"] > bench.issue_bound("60:1", 2.4)["GHs_per_gpu"]


def test_rccl_version_str():
    assert bench.rccl_version_str(22703) == "2.27.3" and bench.rccl_version_str(0) is None


def test_cpu_go_shape_baseline_small(oracle):
    """cpu_baseline.go_shape: the reference loop with hash.go's per-call
    allocations, on a small window; its answer equals the oracle's."""
    lo, hi = 2 ** 32 - (1 << 21), 2 ** 32 - 1
    want = oracle.search(b"bradfitz", lo, hi, threads=4, openssl=True)
    got = bench.cpu_go_shape_baseline(oracle, 4, lo, hi, want, target_s=0.05)
    assert got["result_ok"] and got["value"] > 0 and got["cores"] == 4 and "allocation" in got["kind"], got


def test_c4_block_one_process_and_ranks():
    """bench.c4_block on CPU with a stand-in context: one C4 step over
    [0, 2^40-1] (strong scaling), checked against the committed 2^40 golden,
    per device (one process) or per rank (over a real 2-rank rendezvous in
    test_bench_ranks_join_together's harness; here world 1) with nonces,
    span, rate, start offset and allgather time."""
    from types import SimpleNamespace as NS
    want = bench.golden(b"bradfitz", 0, 2 ** 40 - 1)

    class Ctx:
        calls = []

        def search(self, msg, lo, hi):
            self.calls.append((lo, hi))
            assert msg == b"bradfitz" and 0 <= lo <= hi <= 2 ** 40 - 1
            return tuple(want)

        def last_stats(self):
            half = 2 ** 39
            return NS(nonces=2 ** 40, span_ms=20000.0, combine_used=2, rccl_status=0, rccl_nranks=0, rccl_rank=-1,
                      devices=2, dev_nonces=[half, half], dev_span_ms=[19990.0, 20000.0], dev_rccl_rank=[-1, -1],
                      dev_rccl_device=[-1, -1], rccl_version=22703, rccl_init_ms=0.0, rccl_allgather_ms=0.0,
                      combine_ms=0.02, start_threads=2, dev_start_ms=[0.0, 0.05], dev_allgather_ms=[0.0, 0.0],
                      launches=14)

    ctx = Ctx()
    c4 = bench.c4_block(NS(), ctx, bench.Group(), ctx.search, 2)
    # one tiny untimed search at the start of each of the 13 digit
    # counts first (every C4 layout loaded), then the timed whole range
    assert ctx.calls[-1] == (0, 2 ** 40 - 1) and len(ctx.calls) == 14, ctx.calls
    assert ctx.calls[:2] == [(0, 4095), (10, 4105)] and ctx.calls[12] == (10 ** 12, 10 ** 12 + 4095)
    assert c4["warm"].startswith("13 untimed searches")
    assert (c4["lower"], c4["upper"], c4["nonces"], c4["scaling"]) == (0, 2 ** 40 - 1, 2 ** 40, "strong")
    assert c4["result_ok"] is True and c4["result"] == want and c4["combine"] == "host"
    assert [d["nonces"] for d in c4["devices"]] == [2 ** 39, 2 ** 39] and c4["devices"][1]["start_ms"] == 0.05
    assert c4["GHs"] > 0 and c4["seconds"] >= 0
    # the step record keeps the timed call's launch count (the line's call roofline uses it)
    assert bench.step_record(ctx.last_stats())["launches"] == 14


def test_c4_one_process_block_pieces(monkeypatch):
    """under torchrun, rank 0 measures C4 once more through ONE
    process over the N devices (a child bench.py in the one-process mode).
    On CPU: the child's environment drops the launcher's rank variables; a
    visibility mask that leaves rank 0 fewer than N devices skips the block
    with the reason; the block carries what the verdict asks for from the
    child's line (GH/s, result_ok, per-device nonces / span / start /
    allgather, the combine, rccl_nranks, scaling_valid)."""
    from types import SimpleNamespace as NS
    env = bench.child_env({"RANK": "3", "LOCAL_RANK": "3", "WORLD_SIZE": "8", "TORCHELASTIC_RUN_ID": "x",
                           "LOCAL_WORLD_SIZE": "8", "HIP_VISIBLE_DEVICES": "0,1", "BTCMINER_LIB": "/l.so"})
    assert env == {"WORLD_SIZE": "1", "HIP_VISIBLE_DEVICES": "0,1", "BTCMINER_LIB": "/l.so"}, env
    monkeypatch.setattr(bench, "device_count", lambda: 1)
    blk = bench._c4_one_process_child(NS(rehearse_one_gpu=False, no_balance=False), 2)
    assert "rank 0 sees 1 of 2 devices" in blk["skipped"], blk
    devs = [{"device": i, "pci_bus_id": f"0000:{0x20 + i:02x}:00.0", "nonces": 2 ** 39, "span_ms": 9900.0 + i,
             "GHs": 55.5, "combine": "rccl", "rccl_nranks": 2, "rccl_rank": i, "rccl_device": i,
             "start_ms": 0.01 * i, "allgather_ms": 0.05, "rccl_init_ms": 310.0, "combine_ms": 0.1} for i in range(2)]
    line = {"value": 110.6, "ms_per_step": 9941.0, "steps": 2, "warmup": 1, "result": [16555811, 890536971553],
            "golden": [16555811, 890536971553], "result_ok": True, "rccl_nranks": 2, "scaling_valid": True,
            "rccl": {"version": 22703}, "start_skew_ms": 0.01, "start_threads": 2,
            "config": {"workload": "C4: ...", "lower": 0, "upper": 2 ** 40 - 1, "global_nonces": 2 ** 40,
                       "parallelism": "one process, 2 devices; combine rccl", "devices": devs,
                       "split": {"mode": "measured device rates (bm_ctx_set_balance)", "shares": [65536, 65400]}}}
    blk = bench.one_process_block(line, 2, 25.3, ["--gpus", "2", "--config", "C4"])
    assert blk["GHs"] == 110.6 and blk["result_ok"] is True and blk["combine"] == "rccl", blk
    assert blk["rccl_nranks"] == 2 and blk["scaling_valid"] is True and blk["seconds"] == 9.941
    assert [d["nonces"] for d in blk["devices"]] == [2 ** 39] * 2 and blk["devices"][1]["start_ms"] == 0.01
    assert "bm_ctx_create(2)" in blk["design"] and blk["child_cmd"] == "--gpus 2 --config C4"
    assert "scaling_invalid" not in blk and blk["split"]["shares"] == [65536, 65400]


def test_pmc_same_kernel_code_hash():
    """an imported PMC summary is tied to the kernel it profiled
    by the sha256 of that kernel's instruction bytes in the library's gfx950
    code object (codeobj.py); distinct layouts hash differently, the same
    library twice the same, the clock-probe build (other instructions) not."""
    import pytest
    from distributed_bitcoin_minter_amd import codeobj
    lib = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "libbtcminer.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    c2 = codeobj.kernel_code_sha(lib, 18, 1)
    assert c2 and len(c2) == 64 and c2 == codeobj.kernel_code_sha(lib, 18, 1)
    shas = {codeobj.kernel_code_sha(lib, *k) for k in [(18, 1, 0), (12, 1, 0), (60, 1, 2), (60, 1, 3), (60, 1, 4),
                                                        (13, 2, 0)]}
    assert None not in shas and len(shas) == 6
    assert codeobj.kernel_code_sha(lib, 99, 1) is None
    assert codeobj.mangled_prefix(60, 1, 4) == "_ZN2bm18search_kernel_padkILi60ELi2ELi1EEE"
    probe = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "libbtcminer_probe.so")
    if os.path.exists(probe):
        assert codeobj.kernel_code_sha(probe, 18, 1) not in (None, c2)


def test_wait_exited():
    """bench.wait_exited: rank 0 waits for the other ranks' processes to end
    before the one-process child opens their GPUs; it returns the pids still
    alive at its timeout."""
    import subprocess
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(0.3)"])
    q = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        assert bench.wait_exited([p.pid], timeout_s=20) == []
        p.wait()
        assert bench.wait_exited([q.pid], timeout_s=0.2) == [q.pid]
    finally:
        q.kill()
        q.wait()


# bench.main() itself at world 2 on CPU (VERDICT r5 item 1's sequence): the
# library's Context is a stand-in whose search is the oracle's scan of a small
# range (the group combine stands in with the whole range), the workload and
# the C4 step are shrunk, and the one-process child is replaced by a probe
# that records whether the other ranks are still running when it starts.
_MAIN_WORLD2 = r"""
import json, os, sys, types
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "tests")]
import bench
from conftest import Oracle
from distributed_bitcoin_minter_amd import _lib
from distributed_bitcoin_minter_amd.dist import rank_piece
oracle = Oracle(os.path.join(root, "oracle", "liboracle.so"))
LO, HI = 0, 199_999

def launch(n):
    return types.SimpleNamespace(p=18, nbv=1, pad_block=0, digits=10, inner_digits=2, nonces=n, grid=1792,
                                 tasks_per_thread=1, ms=20.0, clock_ghz=0.0, device=0)

class FakeCtx:
    def __init__(self, devices=None, rank=None, world=None, **kw):
        self.rank_, self.world_, self._joined, self.shares, self.piece = rank, world, False, None, None
    def join(self, uid, timeout_ms=0): self._joined = True
    def joined(self): return self._joined
    def leave(self): self._joined = False
    def set_peer_timeout(self, ms): pass
    def set_timing(self, on): pass
    def num_devices(self): return 1
    def set_split(self, s): self.shares = s
    def close(self): pass
    def search(self, msg, lo, hi):
        self.piece = rank_piece(lo, hi, self.rank_, self.world_, self.shares)
        return oracle.search(msg, lo, hi)   # the in-library allgather: the whole range's answer
    def last_stats(self):
        n = 1 << 31  # as a 2^31-nonce piece would report: the warmup rates are measured on it
        L = launch(n)
        return types.SimpleNamespace(
            nonces=n, span_ms=40.0 + 2 * self.rank_, combine_used=_lib.BM_COMBINED_RCCL, rccl_status=0,
            rccl_nranks=self.world_, rccl_rank=self.rank_, devices=1, dev_nonces=[n], dev_span_ms=[40.0],
            dev_rccl_rank=[self.rank_], dev_rccl_device=[self.rank_], rccl_version=22703, rccl_init_ms=40.0,
            rccl_allgather_ms=0.05, combine_ms=0.2, start_threads=1, dev_start_ms=[0.0], dev_allgather_ms=[0.05],
            launches=1, recorded=1, launch=[L])

rank = int(os.environ["RANK"])
open(os.path.join(os.environ["PIDDIR"], f"pid.{rank}"), "w").write(str(os.getpid()))
bench.Context = FakeCtx
_lib.load = lambda: None
bench.device_count = lambda: 2
bench.rccl_unique_id = lambda: os.urandom(128)
bench.device_pci_bus_id = lambda d: "0000:%02x:00.0" % (0x10 + d)
bench.measure_clock = lambda *a, **k: None
_wl = bench.workload
bench.workload = lambda cfg, n: (b"bradfitz", LO, HI, "weak", "C2 (shrunk for a CPU test)") if cfg == "C2" else _wl(cfg, n)
bench.golden = lambda msg, lo, hi: list(oracle.search(msg, lo, hi)) if hi < 10 ** 6 else None
bench.c4_block = lambda args, ctx, grp, search, n: {"GHs": 1.0, "seconds": 1.0, "result": [0, 0], "golden": None,
                                                  "result_ok": None, "combine": "rccl"}

def probe_child(args, n):
    others = [int(open(os.path.join(os.environ["PIDDIR"], f"pid.{r}")).read()) for r in range(1, 2)]
    return {"GHs": 2.0, "others_running": bench.wait_exited(others, timeout_s=0.0), "n": n}
bench._c4_one_process_child = probe_child
sys.argv = ["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "3", "--no-cpu-baseline", "--clock-sample", "0"]
bench.main()
"""


def test_bench_main_world2_one_process_after_ranks_exit(oracle, tmp_path):
    """bench.main() at world 2 over the file rendezvous, on CPU: the line
    carries the median-of-steps calibration (two warm steps per rank), the
    RCCL block and the ranks; rank 1 exits before rank 0 runs the one-process
    C4 child (the probe sees no other rank running), and only rank 0 prints."""
    import json
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE="2", PIDDIR=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-c", _MAIN_WORLD2, ROOT], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=180) + (p.returncode,) for p in procs]
    assert [rc for _, _, rc in outs] == [0, 0], [e[-2000:] for _, e, _ in outs]
    assert outs[1][0].strip() == ""  # only rank 0 prints the line
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["result_ok"] is True and line["result"] == list(oracle.search(b"bradfitz", 0, 199_999))
    sp = line["config"]["split"]
    assert sp["mode"] == "measured rank rates, median of warmup steps 2..3" and len(sp["step_rates_nonces_per_ms"][0]) == 2
    assert sp["shares"][0] == 65536 and sp["shares"][1] < 65536  # rank 1 reported the longer span
    assert line["rccl"]["version_str"] == "2.27.3" and line["scaling_valid"] is True
    one = line["c4_one_process"]
    assert one["GHs"] == 2.0 and one["n"] == 2 and one["others_running"] == [], one
