#!/usr/bin/env python3
"""Throughput over message lengths: every kernel layout a 10-digit search
reaches, timed on the GPU, with three roofline fractions per layout
(DESIGN.md §5).

For each message length L in 0..max_len (bytes 'a'..), searches of
[10^9, 10^9 + nonces - 1] (all 10-digit, so one layout per L: P, NBV, padding
block).  Per L one JSON line:
  GHs / dom_GHs    the whole call / its dominant launch (HIP events)
  canonical_frac   dom_GHs x C x 1384 / 78.64 T: SURVEY.md §8d's count per
                   compression, C = blocks the kernel compresses per nonce
                   (bench.kernel_compressions).  Not a ceiling: it exceeds 1
                   where constant words fold away
  valu_static      VALU per nonce of the built inner loop (isa_mix.json)
  executed_frac    dom_GHs x VALU per nonce / 78.64 T (static count; with
                   --merge also from PMC: executed_frac_pmc)
  clock_ghz        live shader clock under the dominant launch
                   (libbtcminer_probe.so, s_memtime / s_memrealtime)
  issue_frac       dom_GHs over the loop's issue bound at that clock: the
                   ceiling (bench.issue_bound)
The answers are not checked here (tests/test_gpu_parity.py checks every
layout); this is a measurement.

    python tools/len_sweep.py [--max-len 130] [--nonces 2147483648]      timing sweep (GPU)
    python tools/len_sweep.py --lengths 237-245,1005-1013                 the same over given lengths
        (round 6: the folded padding-block kernels after 3..15 prefix blocks)
    python tools/len_sweep.py --pmc-pass                                  one search per L, prints each
        search's launches; run under BTCMINER_STREAMS=1 BTCMINER_TAIL=0 and
        `rocprofv3 --pmc SQ_INSTS_VALU` (GPU)
    python tools/len_sweep.py --merge SWEEP.jsonl PASS.jsonl COUNTERS.csv  adds VALU per nonce from PMC
        (SQ_INSTS_VALU x 64 / nonces) and executed_frac_pmc to each line (CPU)
"""
import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (roofline helpers; importing it starts nothing)

LO = 10 ** 9


def message(L):
    return bytes(97 + (i % 26) for i in range(L))


def launches_of(st):
    return [st.launch[i] for i in range(st.recorded)]


def lengths(args):
    """0..max_len, or the --lengths spec ("a-b,c,...")."""
    if not args.lengths:
        return list(range(args.max_len + 1))
    out = []
    for part in args.lengths.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def sweep(args):
    from distributed_bitcoin_minter_amd import Context, _lib
    n = args.nonces
    probe = Context(devices=[0], lib_path=_lib.PROBE_LIB_PATH) if os.path.exists(_lib.PROBE_LIB_PATH) else None
    if probe:
        probe.set_timing(True)
    with Context(devices=[0]) as ctx:
        ctx.set_timing(True)
        for L in lengths(args):
            msg = message(L)
            ctx.search(msg, LO, LO + n - 1)  # warm: the layout's code object loads on first launch
            best = None
            for _ in range(2):
                ctx.search(msg, LO, LO + n - 1)
                st = ctx.last_stats()
                if best is None or st.wall_ms < best[0]:
                    dom = max(launches_of(st), key=lambda x: x.nonces)
                    best = (st.wall_ms, dom.p, dom.nbv, dom.pad_block, dom.nonces, dom.ms, st.launches,
                            dom.inner_digits)
            wall, p, nbv, pad, dn, dms, nl, ms = best
            clock = None
            if probe:
                probe.search(msg, LO, LO + n - 1)
                pd = max(launches_of(probe.last_stats()), key=lambda x: x.nonces)
                clock = pd.clock_ghz if pd.clock_ghz > 0 else None
            dom_ghs = dn / dms / 1e6 if dms > 0 else None
            c = 1 + (1 if pad else 0) + (nbv - 1) / 10 ** ms  # NBV = 2: the block before once per task
            line = {"len": L, "P": p, "nbv": nbv, "pad": pad, "launches": nl, "inner_digits": ms,
                    "GHs": round(n / wall / 1e6, 3), "dom_GHs": round(dom_ghs, 3) if dom_ghs else None,
                    "compressions_per_nonce": c}
            if dom_ghs:
                line["canonical_frac"] = round(dom_ghs * 1e9 * c * bench.OPS_PER_COMPRESSION / 1e12 /
                                               bench.VALU_PEAK_T, 4)
                ib = bench.issue_bound(bench.isa_key(p, nbv, pad), clock or 1.0)
                if ib:
                    line["valu_static"] = ib["valu_per_nonce"]
                    line["executed_frac"] = round(dom_ghs * 1e9 * ib["valu_per_nonce"] / 1e12 / bench.VALU_PEAK_T, 4)
                    if clock:
                        line["clock_ghz"] = round(clock, 3)
                        line["executed_frac_live_clock"] = round(line["executed_frac"] * 2.4 / clock, 4)
                        line["issue_bound_GHs"] = ib["GHs_per_gpu"]
                        line["issue_frac"] = round(dom_ghs / ib["GHs_per_gpu"], 4)
            print(json.dumps(line), flush=True)
    if probe:
        probe.close()


def pmc_pass(args):
    """One search per L; its launches in enqueue order (one stream: plan
    order), so rocprof's dispatches can be matched to them."""
    from distributed_bitcoin_minter_amd import Context
    if os.environ.get("BTCMINER_STREAMS") != "1" or os.environ.get("BTCMINER_TAIL") != "0":
        sys.exit("--pmc-pass wants BTCMINER_STREAMS=1 BTCMINER_TAIL=0 (dispatch order = plan order)")
    with Context(devices=[0]) as ctx:
        for L in range(args.max_len + 1):
            ctx.search(message(L), LO, LO + args.nonces - 1)
            st = ctx.last_stats()
            print(json.dumps({"len": L, "launches": [[x.p, x.nbv, x.nonces, x.pad_block] for x in launches_of(st)]}),
                  flush=True)


def merge(sweep_path, pass_path, csv_path):
    """Per layout (P, NBV): SQ_INSTS_VALU x 64 / nonces over the pass's
    search-kernel dispatches, matched in dispatch order to the launches the
    pass printed; added to every sweep line of that layout."""
    valu = collections.defaultdict(float)  # dispatch id -> SQ_INSTS_VALU (summed over its rows)
    names = {}
    for r in csv.DictReader(open(csv_path)):
        if "search_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != "SQ_INSTS_VALU":
            continue
        d = int(r["Dispatch_Id"])
        valu[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    disp = sorted(valu)
    planned = [tuple(x) for ln in open(pass_path) if ln.startswith("{") for x in json.loads(ln)["launches"]]
    if len(planned) != len(disp):
        sys.exit(f"{len(disp)} search-kernel dispatches under PMC, {len(planned)} launches printed by the pass")
    per = collections.defaultdict(lambda: [0.0, 0])  # (P, NBV or "c") -> [VALU lane-ops, nonces]
    for d, (p, nbv, nonces, *pad) in zip(disp, planned):
        kind = bench.isa_key(p, nbv, pad[0] if pad else 0).split(":")[1]  # "c" padc, "kK" padk<P, K>
        name = bench.kernel_name(p, nbv, pad[0] if pad else 0)
        if name not in names[d]:
            sys.exit(f"dispatch {d} is {names[d]}, the pass planned {name}")
        per[(p, kind)][0] += valu[d] * 64
        per[(p, kind)][1] += nonces
    for ln in open(sweep_path):
        if not ln.startswith("{"):
            continue
        line = json.loads(ln)
        v = per.get((line["P"], bench.isa_key(line["P"], line["nbv"], line.get("pad") or 0).split(":")[1]))
        if v and v[1] and line.get("dom_GHs"):
            line["valu_pmc"] = round(v[0] / v[1], 1)
            line["executed_frac_pmc"] = round(line["dom_GHs"] * 1e9 * line["valu_pmc"] / 1e12 / bench.VALU_PEAK_T, 4)
            if line.get("clock_ghz"):
                line["executed_frac_pmc_live_clock"] = round(line["executed_frac_pmc"] * 2.4 / line["clock_ghz"], 4)
        print(json.dumps(line))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-len", type=int, default=130)
    ap.add_argument("--lengths", default=None, help="message lengths instead of 0..max_len, e.g. 237-245,1005-1013")
    ap.add_argument("--nonces", type=int, default=1 << 31)
    ap.add_argument("--pmc-pass", action="store_true")
    ap.add_argument("--merge", nargs=3, metavar=("SWEEP", "PASS", "CSV"))
    args = ap.parse_args()
    if args.merge:
        merge(*args.merge)
    elif args.pmc_pass:
        pmc_pass(args)
    else:
        sweep(args)


if __name__ == "__main__":
    main()
