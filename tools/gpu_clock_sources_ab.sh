#!/bin/bash
# Same box, back to back, alternating: bench.py's sampled driver clock (hwmon
# freq1_input) and the PMC clock under the dominant C2 launch
# (GRBM_GUI_ACTIVE / 8 XCDs / duration).  Which one is the effective clock?
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/clk_bench_$i.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/clk_bench_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('bench',$i,d['value'],'sysfs',r.get('clock_ghz_sysfs'),'kernel_ms',r['kernel_ms'])"
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/clk_pmc_$i -o s --output-format csv -- python3 tools/prof_one.py C2 5 > $OUT/clk_pmc_$i.log 2>&1 || exit $?
  python3 - $OUT/clk_pmc_$i <<'PY'
import csv, collections, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/*counter_collection.csv")[0])))
per = collections.defaultdict(dict); dur = {}
for r in rows:
    if "search_kernel<18, 1>" not in r["Kernel_Name"]:
        continue
    d = r["Dispatch_Id"]; per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print("pmc", [(round(dur[d], 2), round(c["GRBM_GUI_ACTIVE"] / 8 / (dur[d] * 1e-3) / 1e9, 3)) for d, c in per.items()])
PY
done
