#!/usr/bin/env python3
"""A/B of search_kernel_padc (the padding-block layouts of a one-block
message with their constants folded) against the generic padding-block
kernel, on one box, alternating: two contexts in one process, one created
under BTCMINER_PADC=0.  For each message length whose 10-digit nonces end at
byte P >= 55 of block 0 (L = 45..53), REPS alternating searches of
[10^9, 10^9 + nonces - 1] per kernel; prints per length the dominant
launch's rate for each and their ratio, and checks the two answers agree.

    python tools/ab_padc.py [reps] [nonces]        (defaults 5, 2^31)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import Context  # noqa: E402


def dom_rate(ctx):
    st = ctx.last_stats()
    d = max((st.launch[i] for i in range(st.recorded)), key=lambda x: x.nonces)
    return d.nonces / d.ms / 1e6, d.pad_block


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 31
    lo = 10 ** 9
    os.environ["BTCMINER_PADC"] = "0"
    generic = Context(devices=[0])
    del os.environ["BTCMINER_PADC"]
    folded = Context(devices=[0])
    for c in (generic, folded):
        c.set_timing(True)
    summary = []
    for L in range(45, 54):
        msg = bytes(97 + (i % 26) for i in range(L))
        ans = {}
        rates = {"padc": [], "generic": []}
        for name, c in (("padc", folded), ("generic", generic)):
            ans[name] = c.search(msg, lo, lo + n - 1)  # warm
        for _ in range(reps):
            for name, c in (("padc", folded), ("generic", generic)):
                assert c.search(msg, lo, lo + n - 1) == ans[name]
                r, pad = dom_rate(c)
                assert pad == (2 if name == "padc" else 1), (name, pad)
                rates[name].append(r)
        assert ans["padc"] == ans["generic"], (L, ans)
        a = sum(rates["padc"]) / reps
        b = sum(rates["generic"]) / reps
        line = {"len": L, "P": L + 10, "padc_GHs": round(a, 3), "generic_GHs": round(b, 3),
                "ratio": round(a / b, 4), "padc_runs": [round(x, 2) for x in rates["padc"]],
                "generic_runs": [round(x, 2) for x in rates["generic"]], "answer": list(ans["padc"])}
        summary.append(line["ratio"])
        print(json.dumps(line), flush=True)
    print(json.dumps({"mean_ratio": round(sum(summary) / len(summary), 4)}), flush=True)
    generic.close()
    folded.close()


if __name__ == "__main__":
    main()
