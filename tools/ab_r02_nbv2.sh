#!/bin/bash
# NBV = 2 layouts at 7 waves/SIMD (all but P = 4, 13, 14) against the previous
# build (6): parity of the new build, then 50- and 59-byte messages, alternating.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in new; do
  BTCMINER_LIB=$PWD/$D/libbtcminer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)"
done
L="$D/libbtcminer_prev.so $D/libbtcminer.so"
AB_REPS=3 timeout -k 10 900 python -u tools/ab_layouts.py $L $L $L $L > gpurun_out/ab_layouts_nbv2.log 2>&1
echo "ab rc=$?"
