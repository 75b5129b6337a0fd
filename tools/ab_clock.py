#!/usr/bin/env python3
"""Which clock does the C2 call run at, and does bench.py's measure_clock
read the same?  On one box, in one process:
  1. warm, then `reps` C2 calls alternating between the product library
     (no clock stamps) and the clock-probe build (stamps per launch):
     rates of both, and the probe build's in-call live clock of the dominant
     launch;
  2. bench.measure_clock (what the bench line uses for issue_bound: untimed
     searches of the dominant kernel's range after the timed region);
  3. the C2 calls again, as in 1.
Prints one JSON line: rates, in-call clocks before and after, measure_clock's
clock, and the issue-bound fraction each clock gives the product's rate.

    python tools/ab_clock.py [reps]      (default 10)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_bitcoin_minter_amd import Context, _lib  # noqa: E402

MSG, LO, HI = b"bradfitz", 0, (1 << 32) - 1


def phase(prod, probe, reps):
    r = {"prod": [], "probe": [], "clock": []}
    for _ in range(reps):
        for name, c in (("prod", prod), ("probe", probe)):
            t = time.perf_counter()
            c.search(MSG, LO, HI)
            r[name].append((HI - LO + 1) / (time.perf_counter() - t) / 1e9)
            if name == "probe":
                st = c.last_stats()
                dom = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
                r["clock"].append(dom.clock_ghz)
    return {k: sum(v) / len(v) for k, v in r.items()}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    prod = Context(devices=[0])
    probe = Context(devices=[0], lib_path=_lib.PROBE_LIB_PATH)
    for c in (prod, probe):
        c.set_timing(True)
        c.search(MSG, LO, HI)
    a = phase(prod, probe, reps)
    mc = bench.measure_clock(0, MSG, 10, LO, HI, seconds=4.0)
    b = phase(prod, probe, reps)
    prod.close()
    probe.close()
    bound = lambda ghz: bench.issue_bound("18:1", ghz)["GHs_per_gpu"]
    rate = (a["prod"] + b["prod"]) / 2
    incall = (a["clock"] + b["clock"]) / 2
    out = {"prod_GHs": round(rate, 3), "probe_GHs": round((a["probe"] + b["probe"]) / 2, 3),
           "clock_in_call_before": round(a["clock"], 4), "clock_in_call_after": round(b["clock"], 4),
           "measure_clock": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in mc.items()},
           "frac_at_in_call_clock": round(rate / bound(incall), 4),
           "frac_at_measure_clock": round(rate / bound(mc["ghz_live"]), 4) if mc.get("ghz_live") else None}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
