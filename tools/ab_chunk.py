#!/usr/bin/env python3
"""A/B a context-creation knob (default BTCMINER_CHUNK: nonces per lane per
work-counter dequeue; --var BTCMINER_GUIDED ...) on C2 and C3: one process, a
fresh context per setting, settings alternated round after round; best-of-N
wall time, answers checked against the goldens.  Results never depend on the
knob.  The library is BTCMINER_LIB (default: the in-tree build).

    python tools/ab_chunk.py 100 400 1600 [--var BTCMINER_CHUNK] [--rounds 3] [--reps 5]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("chunks", nargs="+", type=int)
ap.add_argument("--var", default="BTCMINER_CHUNK")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
gold = {c["config"]: c for c in json.load(open(os.path.join(ROOT, "tests/golden/full_range.json")))["cases"]}
for rnd in range(a.rounds):
    for ch in a.chunks:
        os.environ[a.var] = str(ch)
        out = {"round": rnd, a.var: ch, "lib": os.path.basename(os.environ.get("BTCMINER_LIB", "libbtcminer.so"))}
        with Context(devices=[0]) as ctx:
            ctx.set_timing(True)
            for cfg in ("C2", "C3"):
                c = gold[cfg]
                msg = bytes.fromhex(c["msg_hex"])
                best = None
                for _ in range(a.reps):
                    assert ctx.search(msg, c["lower"], c["upper"]) == (c["hash"], c["nonce"])
                    st = ctx.last_stats()
                    best = st.wall_ms if best is None else min(best, st.wall_ms)
                dom = max((st.launch[i] for i in range(st.recorded)), key=lambda L: L.nonces)
                out[cfg] = {"wall_ms": round(best, 3), "GHs": round((c["upper"] - c["lower"] + 1) / best / 1e6, 3),
                            "tasks_per_thread": dom.tasks_per_thread}
        print(json.dumps(out), flush=True)
