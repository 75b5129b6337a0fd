#!/usr/bin/env python3
"""Generate the golden fixtures for the nonce-search hot path.

The reference (Go, /root/reference/project2) cannot be built or run here: there
is no Go toolchain and its miner sources do not compile.  Its
arithmetic lives in Go's standard library (crypto/sha256 = FIPS 180-4,
fmt "%s %d", encoding/binary BigEndian; hash.go:3-15), so the vectors are
computed with an independent implementation of the same published function,
Python's hashlib, and anchored on the reference's own known answers
(project2/README.md:331-335).

Outputs (all JSON, small):
  known_answers.json  README:331-335 + README:443 example, recomputed and asserted
  hash_vectors.json   1,000 random (msg, nonce) -> Hash pairs, seed 0x5EED
  search_vectors.json min-scan results over short ranges at block and digit edges
  full_range.json     (--full) C1/C2/C3 whole-range answers from the C oracle
                      (oracle/oracle_cli, 8 threads, OpenSSL block code),
                      whose hashing is first checked against hashlib here.

Usage: python tests/golden/make_golden.py [--full]
"""
import hashlib
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
U64 = (1 << 64) - 1


def ref_hash(msg: bytes, nonce: int) -> int:
    """bitcoin.Hash, hash.go:11-15: sha256(Sprintf("%s %d"))[0:8] big-endian."""
    return int.from_bytes(hashlib.sha256(msg + b" " + str(nonce).encode()).digest()[:8], "big")


def ref_search(msg: bytes, lower: int, upper: int):
    """miner.go:45-46 + :59-65, inclusive upper (README:329)."""
    mh, mn = U64, U64
    for n in range(lower, upper + 1):
        h = ref_hash(msg, n)
        if h < mh:
            mh, mn = h, n
    return mh, mn


def m120() -> bytes:
    return (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]


def known_answers():
    # project2/README.md:333-335 and :331
    ka = {
        "source": "project2/README.md:331-335",
        "hash": [
            {"msg": "msg", "nonce": 0, "hash": 13781283048668101583},
            {"msg": "msg", "nonce": 1, "hash": 4754799531757243342},
            {"msg": "msg", "nonce": 2, "hash": 5611725180048225792},
        ],
        "search": [{"msg": "msg", "lower": 0, "upper": 2, "hash": 4754799531757243342, "nonce": 1}],
    }
    for e in ka["hash"]:
        assert ref_hash(e["msg"].encode(), e["nonce"]) == e["hash"], e
    for e in ka["search"]:
        assert ref_search(e["msg"].encode(), e["lower"], e["upper"]) == (e["hash"], e["nonce"]), e
    # README:443 example input (value computed here, not printed in the README)
    ka["hash"].append({"msg": "thom yorke", "nonce": 19970521,
                       "hash": ref_hash(b"thom yorke", 19970521), "source": "hashlib"})
    return ka


def edge_lengths():
    # msg lengths whose " <digits>" straddle the 55/56/64-byte SHA-256 padding edges
    return [0, 1, 7, 8, 30, 44, 45, 46, 50, 53, 54, 55, 56, 57, 62, 63, 64, 65, 100, 110,
            118, 119, 120, 121, 127, 128, 183, 200, 600]


def make_msg(rng, n):
    alpha = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 .,-_"
    return bytes(rng.choice(alpha) for _ in range(n))


def interesting_nonces(rng):
    out = [0, 1, 9, 10, 99, 100, 12345, 2 ** 32 - 1, 2 ** 32, 10 ** 19 - 1, 10 ** 19, U64 - 1, U64]
    for d in range(1, 21):
        lo = 0 if d == 1 else 10 ** (d - 1)
        hi = min(10 ** d - 1, U64)
        out += [lo, hi, rng.randint(lo, hi)]
    return out


def hash_vectors():
    rng = random.Random(0x5EED)
    vecs = []
    lens = edge_lengths()
    nonces = interesting_nonces(rng)
    for i in range(1000):
        L = lens[i % len(lens)] if i < 600 else rng.randint(0, 300)
        msg = make_msg(rng, L)
        if i % 97 == 0:  # a few raw non-ASCII byte strings: Hash treats msg as bytes
            msg = bytes(rng.randrange(256) for _ in range(L))
        n = nonces[i % len(nonces)] if i % 3 else rng.randint(0, U64)
        vecs.append({"msg_hex": msg.hex(), "nonce": n, "hash": ref_hash(msg, n)})
    return {"seed": "0x5EED", "generator": "hashlib", "vectors": vecs}


def search_vectors():
    rng = random.Random(0x5EED + 1)
    cases = []
    ranges = [(0, 2), (0, 0), (5, 5), (0, 1999), (9990, 10009), (99_999_990, 100_000_009),
              (999_999_000, 1_000_000_999), (2 ** 32 - 700, 2 ** 32 + 300),
              (10 ** 19 - 600, 10 ** 19 + 600), (U64 - 999, U64), (U64, U64),
              (123_456_789_012, 123_456_790_511)]
    for L in edge_lengths():
        msg = make_msg(rng, L)
        for lo, hi in ranges:
            h, n = ref_search(msg, lo, hi)
            cases.append({"msg_hex": msg.hex(), "lower": lo, "upper": hi, "hash": h, "nonce": n})
    # empty range (lower > upper): the loop runs zero times -> (2^64-1, 2^64-1)
    cases.append({"msg_hex": b"msg".hex(), "lower": 10, "upper": 9, "hash": U64, "nonce": U64})
    # the survey's worked cases
    for msg, lo, hi in [(b"bradfitz", 0, 9999), (b"bradfitz", 9990, 10009), (b"bradfitz", U64 - 999, U64),
                        (m120(), U64 - 4095, U64)]:
        h, n = ref_search(msg, lo, hi)
        cases.append({"msg_hex": msg.hex(), "lower": lo, "upper": hi, "hash": h, "nonce": n})
    return {"generator": "hashlib", "bounds": "inclusive", "cases": cases}


def full_range():
    cli = os.path.join(ROOT, "oracle", "oracle_cli")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    # First pin the CLI's OpenSSL path to hashlib on a window of each message.
    for msg, lo, hi in [(b"bradfitz", 2 ** 32 - 3000, 2 ** 32 - 1), (m120(), U64 - 3000, U64)]:
        out = subprocess.check_output([cli, "search", msg.hex(), str(lo), str(hi), "8", "1"]).split()
        assert (int(out[0]), int(out[1])) == ref_search(msg, lo, hi)
    cfgs = [("C1", b"bradfitz", 0, 9999), ("C2", b"bradfitz", 0, 2 ** 32 - 1),
            ("C3", m120(), U64 - (2 ** 32 - 1), U64)]
    res = []
    for name, msg, lo, hi in cfgs:
        out = subprocess.check_output([cli, "search", msg.hex(), str(lo), str(hi), "8", "1"]).split()
        h, n = int(out[0]), int(out[1])
        assert ref_hash(msg, n) == h
        res.append({"config": name, "msg_hex": msg.hex(), "lower": lo, "upper": hi, "hash": h, "nonce": n})
        print(name, h, n, flush=True)
    return {"generator": "oracle/oracle_cli (OpenSSL SHA-256 block code, 8 threads), hash of answer re-checked "
                         "with hashlib", "cases": res}


def main():
    def dump(name, obj):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=0 if name != "hash_vectors.json" else None)
            f.write("\n")

    dump("known_answers.json", known_answers())
    dump("hash_vectors.json", hash_vectors())
    dump("search_vectors.json", search_vectors())
    if "--full" in sys.argv:
        dump("full_range.json", full_range())


if __name__ == "__main__":
    main()
