#!/bin/bash
# A/B of the search kernels' occupancy request on the priority-pass build:
# 8 waves/SIMD (default: 64 VGPRs, 44 B/lane scratch on the C2 kernel's rare
# path), 7 (72 VGPRs, 12 B scratch) and 6 (78 VGPRs, no scratch).  Parity,
# throughput (alternating) and the memory-side write bytes per C2 launch.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
D=distributed_bitcoin_minter_amd
for v in w7 w6; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
for v in default w7 w6; do
  lib=$PWD/$D/libbtcminer.so; [ $v = default ] || lib=$PWD/$D/libbtcminer_$v.so
  BTCMINER_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$v -o w --output-format csv -- python3 tools/prof_one.py C2 2 > $OUT/pmcw_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
  python3 - $OUT/pmcw_$v $v <<'PY'
import csv, collections, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/*counter_collection.csv")[0])))
per = collections.defaultdict(float)
for r in rows:
    if "search_kernel<18, 1>" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
print(sys.argv[2], "WRITE_SIZE KB per <18,1> dispatch:", [round(v) for v in per.values()])
PY
done
L="$D/libbtcminer.so $D/libbtcminer_w7.so $D/libbtcminer_w6.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L > $OUT/ab_waves.log 2>&1
echo "ab rc=$?"
