#!/usr/bin/env python3
"""Golden answers for the long "bradfitz" ranges: the weak-scaling bench
ranges [0, N*2^32-1] (N = 1, 2, 4, 8) and the C4 range [0, 2^40-1].

[0, 2^40-1] is scanned as 256 chunks [k*2^32, (k+1)*2^32-1] by the CPU
oracle's 16-lane AVX-512 scan (oracle/bm_scan16.c, checked against the
byte-string oracle by tests/test_oracle.py).  Every chunk's answer is
re-hashed with hashlib (an independent SHA-256) before it is recorded, and
chunk 0 must equal the C2 whole-range answer in full_range.json, which the
OpenSSL loop of the oracle computed.  The run is resumable: chunk answers
accumulate in c4_chunks.json as they finish (about 20 s each on 8 cores).

The range answers are lexicographic (hash, nonce) minima over chunk answers,
which equal the sequential strict-'<' scan (miner.go:59-65).

Outputs:
  c4_chunks.json    {"chunks": {"k": [hash, nonce]}, ...}  (k = 0..255)
  scale_ranges.json [0, N*2^32-1] for N = 1..8, and C4 once all chunks exist

  c4_windows.json   (--windows) SURVEY §8d(iii): 64 random 2^24-nonce windows of
                    [0, 2^40-1], seed 0x5EED, scanned by the oracle's byte-string
                    loop (OpenSSL block code), not by bm_scan16.c

  c5_clients.json   (--c5) BASELINE C5's 16 client requests: msg "client-%02d",
                    [0, 2^34-1] each, scanned by the AVX-512 scan (answers re-hashed
                    with hashlib)

Usage: python tests/golden/make_chunk_golden.py [--chunks K] [--threads T] [--windows] [--c5]
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

MSG = b"bradfitz"
CHUNK = 1 << 32
NCHUNK = 256  # 2^40 / 2^32
U64 = (1 << 64) - 1


def ref_hash(msg: bytes, nonce: int) -> int:
    """bitcoin.Hash, hash.go:11-15, via hashlib."""
    return int.from_bytes(hashlib.sha256(msg + b" " + str(nonce).encode()).digest()[:8], "big")


def lex_min(pairs):
    best = (U64, U64)
    for p in pairs:
        if tuple(p) < best:
            best = tuple(p)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=NCHUNK, help="compute chunks 0..K-1")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--windows", action="store_true", help="only (re)make c4_windows.json")
    ap.add_argument("--c5", action="store_true", help="only (re)make c5_clients.json")
    args = ap.parse_args()

    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    from conftest import Oracle
    oracle = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))

    if args.c5:
        path = os.path.join(HERE, "c5_clients.json")
        data = json.load(open(path)) if os.path.exists(path) else {
            "config": "C5", "lower": 0, "upper": (1 << 34) - 1, "clients": {}}
        data["generator"] = ("oracle/bm_scan16.c (16-lane AVX-512 scan, checked against oracle_search by "
                             "tests/test_oracle.py); every answer re-hashed with hashlib")
        for i in range(16):
            msg = f"client-{i:02d}"
            if msg in data["clients"]:
                continue
            t = time.time()
            h, n = oracle.search_x16(msg.encode(), 0, (1 << 34) - 1, threads=args.threads)
            assert ref_hash(msg.encode(), n) == h
            data["clients"][msg] = [h, n]
            with open(path + ".tmp", "w") as f:
                json.dump(data, f, indent=0)
                f.write("\n")
            os.replace(path + ".tmp", path)
            print(msg, h, n, f"{time.time() - t:.1f} s", flush=True)
        return

    if args.windows:
        import random
        rng = random.Random(0x5EED)
        wins = []
        for _ in range(64):
            lo = rng.randrange(0, (1 << 40) - (1 << 24) + 1)
            hi = lo + (1 << 24) - 1
            h, n = oracle.search(MSG, lo, hi, threads=args.threads, openssl=True)
            assert lo <= n <= hi and ref_hash(MSG, n) == h
            wins.append({"lower": lo, "upper": hi, "hash": h, "nonce": n})
            print(len(wins), wins[-1], flush=True)
        with open(os.path.join(HERE, "c4_windows.json"), "w") as f:
            json.dump({"msg": MSG.decode(), "seed": "0x5EED", "window": 1 << 24,
                       "generator": "oracle_search_mt (snprintf + OpenSSL SHA-256 per nonce, strict '<'); "
                                    "answers re-hashed with hashlib", "windows": wins}, f, indent=0)
            f.write("\n")
        return

    path = os.path.join(HERE, "c4_chunks.json")
    data = {"msg": MSG.decode(), "chunk": CHUNK, "chunks": {}}
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    data["generator"] = ("oracle/bm_scan16.c (16-lane AVX-512 scan, checked against oracle_search by "
                         "tests/test_oracle.py); every answer re-hashed with hashlib")
    c2 = next(c for c in json.load(open(os.path.join(HERE, "full_range.json")))["cases"] if c["config"] == "C2")

    for k in range(min(args.chunks, NCHUNK)):
        if str(k) in data["chunks"]:
            continue
        lo, hi = k * CHUNK, (k + 1) * CHUNK - 1
        t = time.time()
        h, n = oracle.search_x16(MSG, lo, hi, threads=args.threads)
        assert lo <= n <= hi and ref_hash(MSG, n) == h, (k, h, n)
        if k == 0:
            assert (h, n) == (c2["hash"], c2["nonce"]), "chunk 0 must equal the C2 golden"
        data["chunks"][str(k)] = [h, n]
        with open(path + ".tmp", "w") as f:
            json.dump(data, f, indent=0)
            f.write("\n")
        os.replace(path + ".tmp", path)
        print(f"chunk {k}: [{lo}, {hi}] -> ({h}, {n}) in {time.time() - t:.1f} s", flush=True)

    ch = {int(k): tuple(v) for k, v in data["chunks"].items()}
    out = {"msg_hex": MSG.hex(), "source": "lexicographic min over c4_chunks.json", "ranges": []}
    for N in range(1, 9):
        if all(i in ch for i in range(N)):
            h, n = lex_min(ch[i] for i in range(N))
            out["ranges"].append({"name": f"weak{N}", "lower": 0, "upper": N * CHUNK - 1, "hash": h, "nonce": n})
    if all(i in ch for i in range(NCHUNK)):
        h, n = lex_min(ch.values())
        out["ranges"].append({"name": "C4", "lower": 0, "upper": NCHUNK * CHUNK - 1, "hash": h, "nonce": n})
    with open(os.path.join(HERE, "scale_ranges.json"), "w") as f:
        json.dump(out, f, indent=0)
        f.write("\n")
    print(json.dumps(out["ranges"][-1]))


if __name__ == "__main__":
    main()
