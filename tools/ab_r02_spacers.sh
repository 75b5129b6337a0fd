#!/bin/bash
# A/B of SALU "spacers" in the search kernels' inner loops (round 2): the
# default build (the fold's dead s_mov_b32 kept), those removed (dead), each
# replaced by s_nop 0 (nop), and s_nop 0 between every two adjacent dependent
# VALU (dep).  Parity of each variant first.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in dead nop dep; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)"
done
L="$D/libbtcminer.so $D/libbtcminer_dead.so $D/libbtcminer_nop.so $D/libbtcminer_dep.so"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L $L > gpurun_out/ab_spacers.log 2>&1
echo "ab rc=$?"
