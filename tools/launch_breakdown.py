#!/usr/bin/env python3
"""Per-launch breakdown of one search (HIP-event times from bm_ctx stats):
python tools/launch_breakdown.py [msg] [lower] [upper] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402

msg = (sys.argv[1] if len(sys.argv) > 1 else "bradfitz").encode()
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else (1 << 32) - 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
with Context(devices=[0]) as ctx:
    ctx.set_timing(True)
    ctx.search(msg, lo, hi)
    for _ in range(reps):
        t = time.perf_counter()
        ctx.search(msg, lo, hi)
        wall = (time.perf_counter() - t) * 1e3
        st = ctx.last_stats()
        print(f"wall {wall:.3f} ms (lib {st.wall_ms:.3f}), kernels {st.kernel_ms:.3f} ms, launches {st.launches}")
    for i in range(st.recorded):
        L = st.launch[i]
        print(f"  D={L.digits:2d} P={L.p:2d} nbv={L.nbv} ms_inner={L.inner_digits} nonces={L.nonces:>12d} "
              f"grid={L.grid:5d} {L.ms:9.3f} ms  {L.nonces / max(L.ms, 1e-9) / 1e6:8.2f} GH/s")
