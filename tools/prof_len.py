#!/usr/bin/env python3
"""One search per message length for profiling: python tools/prof_len.py L [L ...]
Each: msg = L bytes 'a'.., nonces [10^9, 10^9 + 2^31 - 1] (the len_sweep
layouts).  PROF_ONE_LAUNCHES=path writes every search's launches (layout,
nonces) in call order, as tools/prof_one.py does."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402

lo = 10 ** 9
launches = []
with Context(devices=[0]) as ctx:
    for L in map(int, sys.argv[1:]):
        msg = bytes(97 + (i % 26) for i in range(L))
        ctx.search(msg, lo, lo + (1 << 31) - 1)
        st = ctx.last_stats()
        launches += [{"len": L, "p": x.p, "nbv": x.nbv, "pad_block": x.pad_block, "nonces": x.nonces}
                     for x in (st.launch[i] for i in range(st.recorded))]
if os.environ.get("PROF_ONE_LAUNCHES"):
    with open(os.environ["PROF_ONE_LAUNCHES"], "w") as f:
        json.dump(launches, f)
print("ok", sys.argv[1:])
