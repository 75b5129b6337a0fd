#!/bin/bash
# On the 7-wave build: are the priority-pass options rejected at 8 waves
# (slow/fast clustering, splitting every 8th add3) still worse?  Parity
# first, then alternating throughput.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in cl s8; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)"
done
L="$D/libbtcminer.so $D/libbtcminer_cl.so $D/libbtcminer_s8.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L > gpurun_out/ab_7wave_passes.log 2>&1
echo "ab rc=$?"
