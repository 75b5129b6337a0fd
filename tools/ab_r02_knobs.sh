#!/bin/bash
# A/B of the launch knobs on the 7-wave build, alternating, the default
# library under each setting: streams 2 (default) / 1 / 3, dequeue chunk 200,
# tail 2^25.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L="BTCMINER_STREAMS=2 BTCMINER_STREAMS=1 BTCMINER_STREAMS=3 BTCMINER_CHUNK=200 BTCMINER_TAIL=33554432"
AB_REPS=5 timeout -k 10 900 python -u tools/ab_bench.py $L $L $L > gpurun_out/ab_knobs.log 2>&1
echo "ab rc=$?"
