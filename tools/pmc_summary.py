#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_*/..._counter_collection.csv)
into profiles/<round>/pmc_summary.json, per kernel: counters summed per
dispatch and averaged over dispatches, HBM bytes per launch
(FETCH_SIZE + WRITE_SIZE, KB -> bytes; MI355X_MICROARCH.md §HBM), the
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and VALU issue rate.
Usage: pmc_summary.py <out_dir> [gpurun_out] [config]
With a config (C2, C3 ...) only the passes under <gpurun_out>/pmc_<config>_*
are read and the summary is written as pmc_summary_<config>.json (what
bench.py looks up for that config's roofline fields).  With the call's
launches (<gpurun_out>/pmc_<config>_launches.json, written by
tools/prof_one.py under PROF_ONE_LAUNCHES) each kernel also gets
valu_per_nonce = SQ_INSTS_VALU x 64 / the nonces of its main launch.
Each kernel also gets code_sha: the sha256 of its instruction bytes in the
library the passes ran (BTCMINER_LIB, else the in-tree libbtcminer.so;
distributed_bitcoin_minter_amd/codeobj.py), so that bench.py can tell whether
an imported summary describes the kernel it loaded (roofline.pmc.same_kernel)."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_bitcoin_minter_amd import codeobj  # noqa: E402

out_dir = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
cfg = sys.argv[3] if len(sys.argv) > 3 else None
per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
dur = collections.defaultdict(dict)
for f in glob.glob(os.path.join(src, f"pmc_{cfg}_*" if cfg else "pmc_*", "*_counter_collection.csv")):
    tag = os.path.basename(os.path.dirname(f))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        d = (tag, r["Dispatch_Id"])
        per[k][d][r["Counter_Name"]] = per[k][d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        dur[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
MIN_CLOCK_S = 0.005  # clock only from launches at least this long
# the profiled call's launches (tools/prof_one.py, PROF_ONE_LAUNCHES): the
# main launch of each kernel layout and its nonces, so SQ_INSTS_VALU becomes
# VALU per nonce (size-independent; bench.py's executed roofline uses it)
main_nonces = {}
lj = os.path.join(src, f"pmc_{cfg}_launches.json") if cfg else None
if lj and os.path.exists(lj):
    for x in json.load(open(lj)):
        name = (f"search_kernel_padc<{x['p']}, 1>" if x["pad_block"] == 2 else
                f"search_kernel_padk<{x['p']}, {x['pad_block'] - 2}, 1>" if x["pad_block"] > 2 else
                f"search_kernel<{x['p']}, {x['nbv']}>")
        main_nonces[name] = max(main_nonces.get(name, 0), x["nonces"])
res = {}
for k, disp in per.items():
    if "search_kernel" not in k:
        continue
    acc, n = collections.defaultdict(list), collections.Counter()
    # main launches only: one template can also run a short tail launch per
    # call, which averaging would mix in
    top = collections.defaultdict(float)
    for d in disp:
        top[d[0]] = max(top[d[0]], dur[k][d])
    for d, cs in disp.items():
        if dur[k][d] <= 0.5 * top[d[0]]:
            continue
        for c, v in cs.items():
            acc[c].append(v)
        acc["_dur_s"].append(dur[k][d])
    m = {c: sum(v) / len(v) for c, v in acc.items()}
    e = {"counters": {c: v for c, v in m.items() if not c.startswith("_")}, "duration_ms": m["_dur_s"] * 1e3}
    for name, nn in main_nonces.items():
        if name + "(" in k and "SQ_INSTS_VALU" in m:
            e["nonces_per_launch"] = nn
            e["valu_per_nonce"] = m["SQ_INSTS_VALU"] * 64 / nn
    lib = os.environ.get("BTCMINER_LIB") or os.path.join(ROOT, "distributed_bitcoin_minter_amd", "libbtcminer.so")
    mk = re.search(r"search_kernel(_padc|_padk)?<(\d+), (\d+)(?:, (\d+))?>", k)
    if mk:
        p, a = int(mk.group(2)), int(mk.group(3))
        kind = mk.group(1)
        nbv, pad = (1, 2) if kind == "_padc" else (1, 2 + a) if kind == "_padk" else (a, 0)
        sha = codeobj.kernel_code_sha(lib, p, nbv, pad)
        if sha:
            e["code_sha"] = sha
            e["code_lib"] = os.path.relpath(lib, ROOT)
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        e["hbm_bytes_per_launch"] = int((m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024)
    if "GRBM_GUI_ACTIVE" in m and m["_dur_s"] >= MIN_CLOCK_S:
        e["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / m["_dur_s"] / 1e9
        if "SQ_INSTS_VALU" in m:
            e["simd_cycles_per_valu"] = (m["GRBM_GUI_ACTIVE"] / 8) * 1024 / m["SQ_INSTS_VALU"]
    elif "GRBM_GUI_ACTIVE" in m:
        # GRBM_GUI_ACTIVE counts the busy cycles of the whole counter window,
        # not only the kernel's: over a launch of a few ms it gave 2.7-6.9 GHz
        e["clock_note"] = f"no clock: launch shorter than {MIN_CLOCK_S * 1e3:.0f} ms"
    res[k] = e
os.makedirs(out_dir, exist_ok=True)
json.dump(res, open(os.path.join(out_dir, f"pmc_summary_{cfg}.json" if cfg else "pmc_summary.json"), "w"), indent=1)
for k, e in res.items():
    print(k[:60], {x: (round(y, 3) if isinstance(y, float) else y) for x, y in e.items() if x != "counters"})
