#!/usr/bin/env python3
"""A/B of library builds over message lengths, on one box, alternating in one
process: the product library and every AB_LIBS="name=path.so ..." build get a
context each; for each length, REPS rounds of one search per context over
[10^9, 10^9 + nonces - 1] (10-digit nonces: one layout per length).  Prints
per length the dominant launch's rate per build and its ratio to the
product's, checks the answers agree, and a mean ratio per build.

    AB_LIBS="v1=a.so v2=b.so" python tools/ab_lens.py 55-60,8 [reps] [nonces]

AB_LO sets the range's start (default 10^9), AB_MAXWIN the planner's window
cap (bm_ctx_set_max_windows; 0 makes every range whose high digits sit in an
earlier block an NBV = 2 launch): e.g. AB_LO=10^15 AB_MAXWIN=0 with L = 61, 62
reaches <13, 2>, <14, 2> (16-digit nonces, 2 and 1 digits in the block before).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402


def lengths(spec):
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    lens = lengths(sys.argv[1] if len(sys.argv) > 1 else "55-60,8")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 31
    lo = int(os.environ.get("AB_LO", 10 ** 9))
    ctxs = [("product", Context(devices=[0]))]
    for spec in os.environ.get("AB_LIBS", "").split():
        name, path = spec.split("=", 1)
        ctxs.append((name, Context(devices=[0], lib_path=os.path.abspath(path))))
    for _, c in ctxs:
        c.set_timing(True)
        if os.environ.get("AB_MAXWIN"):
            c.set_max_windows(int(os.environ["AB_MAXWIN"]))
    ratios = {name: [] for name, _ in ctxs[1:]}
    for L in lens:
        msg = bytes(97 + (i % 26) for i in range(L))
        ans = {name: c.search(msg, lo, lo + n - 1) for name, c in ctxs}  # warm
        assert len(set(ans.values())) == 1, (L, ans)
        rates = {name: [] for name, _ in ctxs}
        for _ in range(reps):
            for name, c in ctxs:
                c.search(msg, lo, lo + n - 1)
                st = c.last_stats()
                d = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
                rates[name].append(d.nonces / d.ms / 1e6)
                layout = (d.p, d.nbv, d.pad_block)
        base = sum(rates["product"]) / reps
        line = {"len": L, "layout": layout, "product_GHs": round(base, 3)}
        for name, _ in ctxs[1:]:
            m = sum(rates[name]) / reps
            line[f"{name}_GHs"] = round(m, 3)
            line[f"{name}_ratio"] = round(m / base, 4)
            ratios[name].append(m / base)
        print(json.dumps(line), flush=True)
    print(json.dumps({f"{k}_mean_ratio": round(sum(v) / len(v), 4) for k, v in ratios.items()}), flush=True)
    for _, c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
