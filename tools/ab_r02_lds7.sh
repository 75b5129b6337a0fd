#!/bin/bash
# A/B on the 7-wave build: a lane's running best in LDS (BM_LDS_BEST=1, no rare-path
# scratch at all) against the default; parity, write bytes per C2 launch, throughput.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
D=distributed_bitcoin_minter_amd
for v in lds; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
for v in default lds; do
  lib=$PWD/$D/libbtcminer.so; [ $v = default ] || lib=$PWD/$D/libbtcminer_$v.so
  BTCMINER_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcl_$v -o w --output-format csv -- python3 tools/prof_one.py C2 2 > $OUT/pmcl_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
  python3 - $OUT/pmcl_$v $v <<'PY'
import csv, collections, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/*counter_collection.csv")[0])))
per = collections.defaultdict(float)
for r in rows:
    if "search_kernel<18, 1>" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
print(sys.argv[2], "WRITE_SIZE KB per <18,1> dispatch:", [round(v) for v in per.values()])
PY
done
L="$D/libbtcminer.so $D/libbtcminer_lds.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L $L > $OUT/ab_lds_7wave.log 2>&1
echo "ab rc=$?"
