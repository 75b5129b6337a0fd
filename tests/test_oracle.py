"""The CPU oracle (oracle/bm_oracle.c) against the golden fixtures.

Pins the oracle before it is trusted as the checker: README:331-335 known
answers, 1,000 hashlib Hash vectors, hashlib min-scan vectors at block and
digit-count edges, and the whole-range answers of C1/C2/C3.
"""
import os
import random

import pytest

from conftest import U64, load_golden


def test_readme_known_answers(oracle):
    ka = load_golden("known_answers.json")
    for e in ka["hash"]:
        assert oracle.hash(e["msg"].encode(), e["nonce"]) == e["hash"]
    for e in ka["search"]:
        assert oracle.search(e["msg"].encode(), e["lower"], e["upper"]) == (e["hash"], e["nonce"])


def test_hash_vectors(oracle):
    for v in load_golden("hash_vectors.json")["vectors"]:
        assert oracle.hash(bytes.fromhex(v["msg_hex"]), v["nonce"]) == v["hash"], v


def test_search_vectors(oracle):
    for c in load_golden("search_vectors.json")["cases"]:
        msg = bytes.fromhex(c["msg_hex"])
        assert oracle.search(msg, c["lower"], c["upper"]) == (c["hash"], c["nonce"]), c
        if c["upper"] - c["lower"] < 3000 and c["lower"] <= c["upper"]:
            assert oracle.search(msg, c["lower"], c["upper"], threads=3) == (c["hash"], c["nonce"])


def test_exclusive_upper_matches_miner_go_loop(oracle):
    # miner.go:59 `for i := Lower; i < Upper; i++`
    msg = b"bradfitz"
    assert oracle.search_excl(msg, 0, 10000) == oracle.search(msg, 0, 9999)
    assert oracle.search_excl(msg, 5, 5) == (U64, U64)


def test_full_range_goldens(oracle):
    """C1 recomputed; C2/C3 answers re-hashed and their neighbourhood
    re-scanned (the whole 2^32 scans take ~1 min each on 8 cores: set
    BM_FULL_ORACLE=1 to recompute them)."""
    full = os.environ.get("BM_FULL_ORACLE") == "1"
    for c in load_golden("full_range.json")["cases"]:
        msg = bytes.fromhex(c["msg_hex"])
        lo, hi, h, n = c["lower"], c["upper"], c["hash"], c["nonce"]
        assert oracle.hash(msg, n) == h
        if c["config"] == "C1" or full:
            assert oracle.search(msg, lo, hi, threads=8, openssl=True) == (h, n)
        else:
            a, b = max(lo, n - 50000), min(hi, n + 50000)
            assert oracle.search(msg, a, b, threads=8) == (h, n)


def test_openssl_and_scalar_agree(oracle):
    """The OpenSSL block code, and the same with hash.go's per-call
    allocations (bench.py's go_shape leg; printf's %llu for the digits),
    equal the scalar restatement, raw bytes and 20-digit nonces included."""
    for msg in (b"The quick brown fox", bytes(range(256)) * 2, b""):
        for lo, hi in [(0, 5000), (U64 - 5000, U64), (999_999_000, 1_000_001_000)]:
            want = oracle.search(msg, lo, hi)
            assert oracle.search(msg, lo, hi, threads=4, openssl=True) == want
            assert oracle.search(msg, lo, hi, threads=3, go_shape=True) == want


def test_x16_scanner_agrees_with_oracle(oracle):
    """The AVX-512 16-lane scan used for the long-range goldens (2^35 weak
    scaling, 2^40 C4) equals the byte-string oracle on every message-length
    class (1 and 2 final blocks, midstate of 0..9 whole blocks), across
    10^k digit boundaries, at 2^64-1, on ranges shorter than 16 lanes and on
    raw bytes."""
    try:
        oracle.search_x16(b"msg", 0, 2)
    except OSError:
        pytest.skip("no AVX-512F on this CPU")
    assert oracle.search_x16(b"msg", 0, 2, threads=1) == (4754799531757243342, 1)  # README:331
    assert oracle.search_x16(b"msg", 5, 4) == (U64, U64)
    rng = random.Random(0x5EED)
    lens = [0, 1, 7, 8, 44, 45, 46, 53, 54, 55, 56, 62, 63, 64, 65, 119, 120, 127, 128, 600]
    for k in range(60):
        L = lens[k % len(lens)] if k < 40 else rng.randint(0, 300)
        msg = bytes(rng.randrange(256) for _ in range(L))
        D = rng.randint(1, 20)
        if k % 3 == 0:  # straddle 10^D
            c = 10 ** D if D < 20 else U64 - 3000
            lo, hi = max(0, c - rng.randint(1, 3000)), min(U64, c + rng.randint(0, 3000))
        else:
            lo = rng.randint(0 if D == 1 else 10 ** (D - 1), U64 if D == 20 else 10 ** D - 1)
            hi = min(U64, lo + rng.choice([0, 1, 5, 15, 16, 17, 999, 5000]))
        want = oracle.search(msg, lo, hi, threads=4)
        assert oracle.search_x16(msg, lo, hi, threads=rng.choice([1, 3, 8])) == want, (L, lo, hi)
    assert oracle.search_x16(b"bradfitz", U64 - 4000, U64) == oracle.search(b"bradfitz", U64 - 4000, U64)
    assert oracle.search_x16(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
