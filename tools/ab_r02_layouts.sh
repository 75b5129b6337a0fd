#!/bin/bash
# Occupancy of the long-message layouts: padding-block layouts at 5 waves/SIMD
# and NBV = 2 at 6 (default) against 4 / 5 (p4) and 6 / 7 (p6).  Parity of
# the variants first, then alternating throughput on 50- and 59-byte messages.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in p4 p6; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)"
done
L="$D/libbtcminer.so $D/libbtcminer_p4.so $D/libbtcminer_p6.so"
AB_REPS=3 timeout -k 10 900 python -u tools/ab_layouts.py $L $L $L > gpurun_out/ab_layouts.log 2>&1
echo "ab rc=$?"
