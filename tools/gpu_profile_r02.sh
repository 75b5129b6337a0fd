#!/bin/bash
# Round-2 GPU evidence in one gpurun call: GPU tests, smoke, bench lines
# (C2 / C3 / C4 at N = 1, the multi-GPU modes rehearsed on one GPU),
# rocprofv3 kernel traces (2 streams and 1 stream) and PMC passes for C2 and
# C3.  Each GPU step has its own time limit; a crash / abort / timeout ends
# the script (rc 1 = pytest "tests failed" is reported and the script goes on).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return $rc
}
TESTS=${TESTS:-1}
if [ "$TESTS" = "1" ]; then
  step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider
fi
step bench_C2 300 python -u bench.py --steps 20 --warmup 5
step bench_C3 300 python -u bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline
step bench_C4_1gpu 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline
step bench_rehearse2_oneproc 300 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 1 --no-cpu-baseline
step bench_rehearse2_torchrun 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 1
step rocprof_C2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2
export BTCMINER_STREAMS=1
step rocprof_C2_1stream 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C2_1stream -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2
unset BTCMINER_STREAMS
step rocprof_C3 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C3 -o run --output-format csv -- python3 bench.py --config C3 --no-cpu-baseline --steps 5 --warmup 2
for C in C2 C3; do
  step pmc_${C}_fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_${C}_fetch -o f --output-format csv -- python3 tools/prof_one.py $C 2
  step pmc_${C}_write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_${C}_write -o w --output-format csv -- python3 tools/prof_one.py $C 2
  step pmc_${C}_sq 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $OUT/pmc_${C}_sq -o s --output-format csv -- python3 tools/prof_one.py $C 2
done
echo done
