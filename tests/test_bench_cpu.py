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
