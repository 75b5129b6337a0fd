#!/bin/bash
# Is the search kernel issue-bound or power-bound?  Variants that move slow
# VALU into the fast class (split every 8th / 4th all-VGPR v_add3: issue bound
# -2.3% / -0.9% slots per nonce) against the default build: throughput A/B
# (alternating) and, per variant, the clock under the C2 kernel from PMC
# (GRBM_GUI_ACTIVE / 8 XCDs / duration, tools/pmc_summary.py).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
D=distributed_bitcoin_minter_amd
for v in s8 s4; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
for v in default s8 s4 default; do
  lib=$PWD/$D/libbtcminer.so; [ $v = default ] || lib=$PWD/$D/libbtcminer_$v.so
  BTCMINER_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmcclk_$v -o s --output-format csv -- python3 tools/prof_one.py C2 3 > $OUT/pmcclk_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
  echo "pmc $v ok"
done
L="$D/libbtcminer.so $D/libbtcminer_s8.so $D/libbtcminer_s4.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L > $OUT/ab_split_clock.log 2>&1
echo "ab rc=$?"
