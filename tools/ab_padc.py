#!/usr/bin/env python3
"""A/B of search_kernel_padc (the padding-block layouts of a one-block
message with their constants folded) against the generic padding-block
kernel, on one box, alternating: two contexts in one process, one created
under BTCMINER_PADC=0.  For each message length whose 10-digit nonces end at
byte P >= 55 of block 0 (L = 45..53), REPS alternating searches of
[10^9, 10^9 + nonces - 1] per kernel; prints per length the dominant
launch's rate for each and their ratio, and checks the two answers agree.

    python tools/ab_padc.py [reps] [nonces]        (defaults 5, 2^31)

AB_LIBS="name=path.so ..." adds one more context per library build (e.g. a
build with another bm_prio.py option or kernel macro), alternating with the
two above; ratios are against the generic kernel of the product library.
AB_LENS="109-117" sweeps other message lengths: there the messages have one
prefix block, which the default context runs with search_kernel_padk<P, 1>
since round 5, and "173-181" two (search_kernel_padk<P, 2>).
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
    ctxs = [("generic", Context(devices=[0]))]
    del os.environ["BTCMINER_PADC"]
    ctxs.append(("padc", Context(devices=[0])))
    for spec in os.environ.get("AB_LIBS", "").split():
        name, path = spec.split("=", 1)
        ctxs.append((name, Context(devices=[0], lib_path=os.path.abspath(path))))
    for _, c in ctxs:
        c.set_timing(True)
    summary = {name: [] for name, _ in ctxs[1:]}
    a, b = map(int, os.environ.get("AB_LENS", "45-53").split("-"))
    for L in range(a, b + 1):
        msg = bytes(97 + (i % 26) for i in range(L))
        ans = {name: c.search(msg, lo, lo + n - 1) for name, c in ctxs}  # warm
        rates = {name: [] for name, _ in ctxs}
        pads = {}
        for _ in range(reps):
            for name, c in ctxs:
                assert c.search(msg, lo, lo + n - 1) == ans[name]
                r, pad = dom_rate(c)
                assert pad >= 1 and (name != "generic" or pad == 1), (name, pad)
                pads[name] = pad
                rates[name].append(r)
        assert len(set(ans.values())) == 1, (L, ans)
        base = sum(rates["generic"]) / reps
        line = {"len": L, "P": (L + 10) % 64, "pad_block": pads, "answer": list(ans["generic"])}
        for name, _ in ctxs:
            m = sum(rates[name]) / reps
            line[f"{name}_GHs"] = round(m, 3)
            line[f"{name}_runs"] = [round(x, 2) for x in rates[name]]
            if name != "generic":
                line[f"{name}_ratio"] = round(m / base, 4)
                summary[name].append(m / base)
        print(json.dumps(line), flush=True)
    print(json.dumps({f"{k}_mean_ratio": round(sum(v) / len(v), 4) for k, v in summary.items()}), flush=True)
    for _, c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
