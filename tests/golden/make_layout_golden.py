#!/usr/bin/env python3
"""Full-size golden answers for the padding-block and straddling layouts
(round 4: search_kernel_padc, the generic padding-block kernel's add3_sgpr,
NBV = 2): for a few message lengths, the whole 2^32-nonce 10-digit range
[10^9, 10^9 + 2^32 - 1], scanned by the CPU oracle's 16-lane AVX-512 scan
(oracle/bm_scan16.c; test infrastructure).  Before each long scan the
scanner is checked against the oracle's byte-string loop (OpenSSL block
code) on a 2^21-nonce window of the same message, and every answer's hash is
re-computed with hashlib (an independent SHA-256).

Messages are L bytes 'a'.. (tools/len_sweep.py's); lengths:
  50  last digit at byte 60 of block 0: padding block, search_kernel_padc
  46  byte 56 of block 0 (P % 4 = 0): padc with the two-word inner loop
  114 byte 60 of block 1: padding block after a prefix block (the generic kernel
      until round 4; search_kernel_padk<60, 1> since round 5)
  178 byte 60 of block 2: padding block after two prefix blocks, search_kernel_padk<60, 2>
  242 byte 60 of block 3: after three prefix blocks, search_kernel_padk<60, 3> (round 6)
  1010 byte 60 of block 15: after fifteen, search_kernel_padk<60, 15> (round 6: the
      largest folded K, a message of about an LSP packet's 1,000 bytes)
  59  digits straddle blocks 0 and 1: NBV = 2

Usage: python tests/golden/make_layout_golden.py [--threads T] [--lengths 178 ...]
       (about a minute per length on 8 cores; --lengths recomputes only those and keeps the others)
"""
import argparse
import hashlib
import json
import os
import subprocess
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CLI = os.path.join(ROOT, "oracle", "oracle_cli")
LENGTHS = {50: "padc", 46: "padc, two-word inner loop", 114: "padding block after one prefix block",
           59: "NBV = 2", 178: "padding block after two prefix blocks",
           242: "padding block after three prefix blocks", 1010: "padding block after fifteen prefix blocks"}
LO = 10 ** 9
HI = LO + (1 << 32) - 1


def message(L):
    return bytes(97 + (i % 26) for i in range(L))


def ref_hash(msg, n):
    return int.from_bytes(hashlib.sha256(msg + b" " + str(n).encode()).digest()[:8], "big")


def scan(kind, msg, lo, hi, threads):
    args = [CLI, kind, msg.hex(), str(lo), str(hi), str(threads)] + (["1"] if kind == "search" else [])
    h, n = map(int, subprocess.check_output(args).split()[:2])
    return h, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--lengths", type=int, nargs="*", default=None)
    a = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    path = os.path.join(HERE, "layout_ranges.json")
    old = {c["len"]: c for c in json.load(open(path))["cases"]} if a.lengths and os.path.exists(path) else {}
    cases = []
    for L, what in LENGTHS.items():
        if a.lengths and L not in a.lengths and L in old:
            cases.append(dict(old[L], layout=what))
            continue
        msg = message(L)
        w = (HI - (1 << 21) + 1, HI)
        assert scan("search16", msg, *w, a.threads) == scan("search", msg, *w, a.threads), L
        t = time.time()
        h, n = scan("search16", msg, LO, HI, a.threads)
        assert ref_hash(msg, n) == h and LO <= n <= HI, L
        cases.append({"len": L, "layout": what, "msg_hex": msg.hex(), "lower": LO, "upper": HI, "hash": h, "nonce": n})
        print(L, what, h, n, f"{time.time() - t:.0f} s", flush=True)
    with open(path, "w") as f:
        json.dump({"generator": "oracle/oracle_cli search16 (AVX-512), checked against the OpenSSL loop on a "
                                "2^21 window per message; answers re-hashed with hashlib", "cases": cases}, f, indent=0)
        f.write("\n")


if __name__ == "__main__":
    main()
