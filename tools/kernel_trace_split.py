#!/usr/bin/env python3
"""Per-launch view of a rocprofv3 kernel trace (run_kernel_trace.csv) for the
search kernels.  With two launch streams and the tail launch
one template can run twice per call (main piece + 2^24-nonce tail piece), so
rocprof's per-name average mixes the two; this splits them by duration and
reports the main launch's average, which is what bench.py's roofline.kernel_ms
measures with HIP events.

    python tools/kernel_trace_split.py gpurun_out/prof/run_kernel_trace.csv > profiles/r01/bench_kernel_split.json
"""
import collections
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "search_kernel" in r["Kernel_Name"]]
by = collections.defaultdict(list)
ids = collections.defaultdict(lambda: collections.defaultdict(list))  # name -> Kernel_Id -> durations
for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ids[name][r["Kernel_Id"]].append(d)
# One Kernel_Id per loaded code object: a process that loads two builds of
# the library (bench.py's clock measurement uses libbtcminer_probe.so after
# its timed region) has two ids per template; the first one dispatched is the
# product library's, and it is what the per-name figures below describe.
out_ids = {}
for name, per in ids.items():
    order = list(per)  # dispatch order of first appearance
    by[name] = per[order[0]]
    if len(order) > 1:
        out_ids[name] = {k: {"calls": len(v), "max_ms": round(max(v), 3)} for k, v in per.items()}
# Main launches: the cluster around the median of the longer half of a
# template's launches (the timed steps' main pieces); shorter ones are the
# tail pieces and other calls' small launches; much longer ones (>= 2x) are
# other calls' big launches -- since round 5 every bench line ends with a C4
# step, whose 10-digit launch of the same template runs 9e9 nonces while its
# other stream's launches stretch it, and which must not count as a main one.
out = {}
for name, ds in sorted(by.items(), key=lambda kv: -max(kv[1])):
    top_half = sorted(ds)[len(ds) // 2:]
    ref = top_half[len(top_half) // 2]
    main = [d for d in ds if 0.5 * ref < d < 2 * ref]
    rest = [d for d in ds if d <= 0.5 * ref]
    big = [d for d in ds if d >= 2 * ref]
    out[name] = {"calls": len(ds), "main_calls": len(main), "main_avg_ms": round(sum(main) / len(main), 3),
                 "other_calls": len(rest), "other_avg_ms": round(sum(rest) / len(rest), 3) if rest else None}
    if big:
        out[name]["long_calls"] = len(big)
        out[name]["long_ms"] = [round(d, 3) for d in big]
if out_ids:
    out["_kernel_ids"] = {"note": "templates dispatched from more than one code object; the entries above use "
                                  "the first (the product library)", "ids": out_ids}
json.dump(out, sys.stdout, indent=1)
print()
