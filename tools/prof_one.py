#!/usr/bin/env python3
"""Run ONE C2 search (and optionally C3) for profiling: python tools/prof_one.py [C2|C3] [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context
cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = {c["config"]: c for c in json.load(open(os.path.join(ROOT, "tests/golden/full_range.json")))["cases"]}[cfg]
with Context(devices=[0]) as ctx:
    for _ in range(reps):
        r = ctx.search(bytes.fromhex(c["msg_hex"]), c["lower"], c["upper"])
        assert r == (c["hash"], c["nonce"]), r
    # PROF_ONE_LAUNCHES=path: the last call's launches (kernel layout, nonces),
    # so tools/pmc_summary.py can turn a counter per dispatch into one per nonce
    if os.environ.get("PROF_ONE_LAUNCHES"):
        st = ctx.last_stats()
        with open(os.environ["PROF_ONE_LAUNCHES"], "w") as f:
            json.dump([{"p": x.p, "nbv": x.nbv, "pad_block": x.pad_block, "nonces": x.nonces}
                       for x in (st.launch[i] for i in range(st.recorded))], f)
print("ok", cfg, r)
