#!/bin/bash
# A/B of the search kernels' workgroup size on the 7-wave build: 256 threads
# (default) against 64, 128 and 512 (BM_BLOCK).  Parity first.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in b64 b128 b512; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -q -x -k "not bench and not c4_whole" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)"
done
L="$D/libbtcminer.so $D/libbtcminer_b64.so $D/libbtcminer_b128.so $D/libbtcminer_b512.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L > gpurun_out/ab_block.log 2>&1
echo "ab rc=$?"
