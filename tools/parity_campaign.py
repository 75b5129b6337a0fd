#!/usr/bin/env python3
"""Randomized GPU-vs-oracle parity campaign (longer than the pytest suite):

    python tools/parity_campaign.py [cases] [seed]

Each case: a random raw-byte message (0..1,100 bytes, any byte value: since
round 6 past the 1,024-byte reach of the folded padding kernels), a random
digit class 1..20, a random window of 1..2^22 nonces inside it (clipped at
2^64-1), and sometimes a window that straddles a power of ten.  Task size and
planner window cap are randomized too.  Kernels are counted per layout, the
folded padding-block kernels (search_kernel_padc, search_kernel_padk<P, K>:
stats pad_block = 2 + K) apart from search_kernel.  bm_search_gpu must equal the CPU
oracle's sequential scan (hash.go:11-15 + miner.go:59-65, inclusive bounds)
bit for bit.  Prints one JSON summary line; exits 1 on the first mismatch.
The oracle is the checker only (test infrastructure)."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import Oracle  # noqa: E402
from distributed_bitcoin_minter_amd import Context  # noqa: E402

U64 = (1 << 64) - 1


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0x5EED
    rng = random.Random(seed)
    oracle = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    nonces = 0
    t0 = time.perf_counter()
    layouts = set()
    folded = {}  # pad_block (2 + K) -> launches of the folded padding-block kernels
    with Context(devices=[0]) as ctx:
        for i in range(cases):
            L = rng.choice([rng.randint(0, 130), rng.randint(0, 700), rng.randint(0, 1100)])
            msg = bytes(rng.randrange(256) for _ in range(L))
            D = rng.randint(1, 20)
            dlo = 0 if D == 1 else 10 ** (D - 1)
            dhi = U64 if D == 20 else 10 ** D - 1
            width = rng.randint(1, 1 << rng.randint(0, 22))
            if rng.random() < 0.2 and D < 20:  # straddle 10^D
                lo = max(0, 10 ** D - rng.randint(1, width))
            else:
                lo = rng.randint(dlo, dhi)
            hi = min(U64, lo + width - 1)
            ctx.set_task_digits(rng.choice([0, 0, 1, 2]))
            ctx.set_max_windows(rng.choice([64, 64, 0, 3]))
            got = ctx.search(msg, lo, hi)
            want = oracle.search(msg, lo, hi, threads=threads)
            st = ctx.last_stats()
            for k in range(st.recorded):
                pb = st.launch[k].pad_block
                layouts.add((st.launch[k].nbv, st.launch[k].p, pb if pb >= 2 else 0))
                if pb >= 2:
                    folded[pb] = folded.get(pb, 0) + 1
            nonces += hi - lo + 1
            if got != want:
                print(json.dumps({"ok": False, "case": i, "msg_hex": msg.hex(), "lower": lo, "upper": hi,
                                  "got": list(got), "want": list(want)}), flush=True)
                return 1
            if (i + 1) % 200 == 0:
                print(f"{i + 1} cases ok, {nonces} nonces, {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    print(json.dumps({"ok": True, "cases": cases, "seed": seed, "nonces": nonces, "layouts_hit": len(layouts),
                      "padc_layouts_hit": sum(1 for x in layouts if x[2] == 2),
                      "padk_layouts_hit": {f"K={pb - 2}": sum(1 for x in layouts if x[2] == pb) for pb in range(3, 18)},
                      "folded_launches": {f"K={pb - 2}": n for pb, n in sorted(folded.items())},
                      "seconds": round(time.perf_counter() - t0, 1), "oracle_threads": threads}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
