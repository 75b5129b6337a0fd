#!/bin/bash
# Round-2 (second session) GPU evidence in one gpurun call: smoke, the GPU
# suite, bench lines (C2, C3), rocprofv3 kernel traces (2 streams, 1 stream),
# one PMC pass per block for C2, and an A/B of the dead-s_mov build against
# the default one (parity first).  Each GPU step has its own time limit; a
# crash / abort / timeout ends the script (rc 1 = pytest "tests failed" is
# reported and the script goes on).
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
D=distributed_bitcoin_minter_amd
if [ "${TESTS:-1}" = "1" ]; then
  step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
  step gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
step bench_C2 300 python -u bench.py --steps 20 --warmup 5
step bench_C3 300 python -u bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline
step rocprof_C2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2
export BTCMINER_STREAMS=1
step rocprof_C2_1stream 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C2_1stream -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2
unset BTCMINER_STREAMS
step pmc_C2_fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_C2_fetch -o f --output-format csv -- python3 tools/prof_one.py C2 2
step pmc_C2_write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_C2_write -o w --output-format csv -- python3 tools/prof_one.py C2 2
step pmc_C2_sq 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $OUT/pmc_C2_sq -o s --output-format csv -- python3 tools/prof_one.py C2 2
if [ -f $D/libbtcminer_dead.so ]; then
  BTCMINER_LIB=$PWD/$D/libbtcminer_dead.so step parity_dead 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
  [ $? -eq 0 ] || { echo "parity_dead failed"; exit 1; }
  L="$D/libbtcminer.so $D/libbtcminer_dead.so"
  AB_REPS=5 step ab_dead_smov 600 python -u tools/ab_bench.py $L $L $L $L
fi
echo done
