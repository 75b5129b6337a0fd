#!/usr/bin/env python3
"""What one bm_search_gpu call costs at each size: GH/s
of whole calls over ranges of 2^24 .. 2^34 nonces, on one device and on a
context of N slots (default 8) all on GPU 0 -- the latter adds what an
N-device context adds per call (N submission threads, N plans, the combine;
host copies here, since RCCL refuses one GPU twice), not N GPUs' work.

Every range is 'bradfitz' starting at 10^10 (11-digit nonces, one layout
throughout, <19, 1>: the same loop as C2's <18, 1> one byte later), so the
curve isolates the per-call cost.  Each size is called at least `--reps`
times and for at least `--min-s` seconds; the rate is nonces / mean wall time
per call (host wall clock around the synchronous call).  `eff` is that rate
over the largest size's on the same context.

    python tools/call_size.py [--slots 8] [--min-bits 24] [--max-bits 34] [--out f.json] [--lib other.so]

The server sizes jobs from this: a job of about 0.3 s is within 1% of the
asymptotic rate."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402

MSG = b"bradfitz"
LO = 10 ** 10


def curve(ctx, bits, reps, min_s):
    out = []
    for b in bits:
        n = 1 << b
        ctx.search(MSG, LO, LO + n - 1)  # warm (first launch of the layout, plan caches)
        k, t = 0, time.perf_counter()
        while k < reps or time.perf_counter() - t < min_s:
            ctx.search(MSG, LO, LO + n - 1)
            k += 1
        dt = (time.perf_counter() - t) / k
        out.append({"bits": b, "nonces": n, "calls": k, "ms_per_call": round(dt * 1e3, 4),
                    "GHs": round(n / dt / 1e9, 3)})
        print(json.dumps(out[-1]), flush=True)
    top = out[-1]["GHs"]
    for e in out:
        e["eff"] = round(e["GHs"] / top, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--min-bits", type=int, default=24)
    ap.add_argument("--max-bits", type=int, default=34)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--min-s", type=float, default=1.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="another build of the library (an A/B)")
    a = ap.parse_args()
    bits = list(range(a.min_bits, a.max_bits + 1))
    res = {"msg": MSG.decode(), "lower": LO, "note": __doc__.split("\n\n")[0], "lib": a.lib or "libbtcminer.so"}
    kw = {"lib_path": os.path.abspath(a.lib)} if a.lib else {}
    with Context(devices=[0], **kw) as c:
        print("== one device", flush=True)
        res["one_device"] = curve(c, bits, a.reps, a.min_s)
    with Context(devices=[0] * a.slots, **kw) as c:
        print(f"== {a.slots} slots on GPU 0 (host combine)", flush=True)
        res[f"slots_{a.slots}_on_gpu0"] = curve(c, bits, a.reps, a.min_s)
        st = c.last_stats()
        res["start_threads"] = st.start_threads
    for name in ("one_device", f"slots_{a.slots}_on_gpu0"):
        print(name, " ".join(f"2^{e['bits']}:{e['eff']:.3f}" for e in res[name]), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
