#!/usr/bin/env python3
"""Throughput over message lengths: every kernel layout a 10-digit search
reaches, timed on the GPU.

    python tools/len_sweep.py [max_len] [nonces]        (defaults 130, 2^31)

For each message length L in 0..max_len (bytes 'a'..), one search of
[10^9, 10^9 + nonces - 1] (all 10-digit, so one layout per L: P, NBV, padding
block) after a warm-up call; prints one JSON line per L with GH/s and the
compressions the kernel does per nonce (1, + the padding block, + 1/task for
NBV = 2), so layouts can
be compared per compression: G compressions/s should sit near the C2 figure
for every layout.  The answers are not checked here (tests/test_gpu_parity.py
checks every layout); this is a measurement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402


def main():
    max_len = int(sys.argv[1]) if len(sys.argv) > 1 else 130
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 31
    lo = 10 ** 9
    with Context(devices=[0]) as ctx:
        ctx.set_timing(True)
        for L in range(max_len + 1):
            msg = bytes(97 + (i % 26) for i in range(L))
            ctx.search(msg, lo, lo + n - 1)  # warm: the layout's code object loads on first launch
            best = None
            for _ in range(2):
                ctx.search(msg, lo, lo + n - 1)
                st = ctx.last_stats()
                if best is None or st.wall_ms < best[0]:
                    dom = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
                    best = (st.wall_ms, dom.p, dom.nbv, dom.pad_block, dom.nonces, dom.ms, st.launches, dom.inner_digits)
            wall, p, nbv, pad, dn, dms, nl, ms = best
            c = 1 + pad + (nbv - 1) / 10 ** ms  # NBV = 2: the block before once per task
            print(json.dumps({"len": L, "P": p, "nbv": nbv, "pad": pad, "launches": nl,
                              "GHs": round(n / wall / 1e6, 3), "Gcomp_s": round(c * n / wall / 1e6, 3),
                              "dom_GHs": round(dn / dms / 1e6, 3) if dms > 0 else None}), flush=True)


if __name__ == "__main__":
    main()
