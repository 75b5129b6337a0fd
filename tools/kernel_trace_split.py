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
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for name, ds in sorted(by.items(), key=lambda kv: -max(kv[1])):
    top = max(ds)
    main = [d for d in ds if d > 0.5 * top]
    rest = [d for d in ds if d <= 0.5 * top]
    out[name] = {"calls": len(ds), "main_calls": len(main), "main_avg_ms": round(sum(main) / len(main), 3),
                 "other_calls": len(rest), "other_avg_ms": round(sum(rest) / len(rest), 3) if rest else None}
json.dump(out, sys.stdout, indent=1)
print()
