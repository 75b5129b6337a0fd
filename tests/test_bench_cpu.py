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
