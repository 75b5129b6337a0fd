#!/bin/bash
# What the driver runs at round end, in its own words: the GPU suite, smoke(),
# and the default bench line.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 700 python -m pytest tests/ -x -q -m gpu > $OUT/driver_gpu_tests.log 2>&1; rc=$?; tail -1 $OUT/driver_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/driver_smoke.log 2>&1 || exit $?
tail -1 $OUT/driver_smoke.log
timeout -k 10 400 python bench.py > $OUT/driver_bench.json 2> $OUT/driver_bench.err || exit $?
cut -c1-200 $OUT/driver_bench.json
