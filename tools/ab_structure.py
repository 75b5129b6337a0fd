#!/usr/bin/env python3
"""Does C2's multi-launch structure cost throughput?  Alternates, in one
process on the clock-probe build (every launch stamps its own shader clock):
  C2     'bradfitz' [0, 2^32-1]: 11 launches (1- to 10-digit segments + tail)
  D10    'bradfitz' [10^9, 10^9 + 2^32 - 1]: the same 2^32 nonces, all 10-digit
         (one main launch + tail)
and prints, per call, nonces / wall and that rate over the issue bound at the
dominant launch's live clock (isa_mix.json's slots for <18, 1>), so a gap
between the two is the cost of the small segments and their ordering.

    python tools/ab_structure.py [reps]      (default 8)
Env BTCMINER_STREAMS / BTCMINER_TAIL apply as usual (read at context creation).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_bitcoin_minter_amd import Context, _lib  # noqa: E402

WORK = {"C2": (0, (1 << 32) - 1), "D10": (10 ** 9, 10 ** 9 + (1 << 32) - 1)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    path = _lib.PROBE_LIB_PATH if os.path.exists(_lib.PROBE_LIB_PATH) else None
    res = {k: [] for k in WORK}
    with Context(devices=[0], lib_path=path) as ctx:
        ctx.set_timing(True)
        for lo, hi in WORK.values():
            ctx.search(b"bradfitz", lo, hi)  # warm
        for _ in range(reps):
            for name, (lo, hi) in WORK.items():
                t = time.perf_counter()
                ctx.search(b"bradfitz", lo, hi)
                wall = time.perf_counter() - t
                st = ctx.last_stats()
                dom = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
                ib = bench.issue_bound(bench.isa_key(dom.p, dom.nbv, dom.pad_block), dom.clock_ghz) if dom.clock_ghz > 0 else None
                rate = (hi - lo + 1) / wall / 1e9
                res[name].append({"GHs": rate, "span_GHs": (hi - lo + 1) / st.span_ms / 1e6,
                                  "clock": dom.clock_ghz, "launches": st.launches,
                                  "frac_wall": rate / ib["GHs_per_gpu"] if ib else None,
                                  "frac_span": (hi - lo + 1) / st.span_ms / 1e6 / ib["GHs_per_gpu"] if ib else None})
    out = {"probe_build": bool(path), "streams": os.environ.get("BTCMINER_STREAMS", "default"),
           "tail": os.environ.get("BTCMINER_TAIL", "default")}
    for name, rs in res.items():
        m = lambda k: round(sum(r[k] for r in rs) / len(rs), 4) if all(r[k] is not None for r in rs) else None
        out[name] = {k: m(k) for k in ("GHs", "span_GHs", "clock", "frac_wall", "frac_span")}
        out[name]["launches"] = rs[-1]["launches"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
