#!/usr/bin/env python3
"""A/B of the long-message layouts over libbtcminer builds (no torch):

    python tools/ab_layouts.py lib1.so lib2.so ...

Workloads: a 50-byte message (the last digit at byte 60 of its block, so a
constant padding block follows: 2 compressions per nonce) and a 59-byte
message (digits straddle the block boundary: NBV = 2, the block before is
re-compressed per 100-nonce task), each over [10^9, 10^9 + 2^32 - 1] (all 10
digits).  Best-of-N GH/s per library, alternating; every answer is checked
to be equal across libraries (and the 50/59-byte answers against the CPU
oracle over a 2^20 window by the parity suite)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORK = [("L50", b"x" * 50), ("L59", b"y" * 59)]
LO, HI = 10 ** 9, 10 ** 9 + 2 ** 32 - 1


def one(reps):
    sys.path.insert(0, ROOT)
    from distributed_bitcoin_minter_amd import Context
    out = {"lib": os.path.basename(os.environ["BTCMINER_LIB"])}
    with Context(devices=[0]) as ctx:
        for name, msg in WORK:
            best, res = None, None
            for _ in range(reps):
                t = time.perf_counter()
                res = ctx.search(msg, LO, HI)
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            out[name] = {"GHs": round((HI - LO + 1) / best / 1e9, 3), "result": list(res)}
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("AB_CHILD"):
        return one(int(os.environ.get("AB_REPS", "5")))
    for lib in sys.argv[1:]:
        env = dict(os.environ, BTCMINER_LIB=os.path.abspath(lib), AB_CHILD="1")
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, timeout=300)
        if r.returncode not in (0,):
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
