#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# script (exit codes other than 0 and 1 = pytest "tests failed").
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return $rc
}
rocminfo 2>/dev/null | grep -m1 -E "gfx9[0-9]+" > $OUT/arch.txt; cat $OUT/arch.txt
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step bench 300 python -u bench.py
cp $OUT/bench.log $OUT/bench.json 2>/dev/null
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline
fi
if [ "${PMC:-1}" = "1" ]; then
  step pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 tools/prof_one.py C2
  step pmc_write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 tools/prof_one.py C2
  step pmc_sq 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o s --output-format csv -- python3 tools/prof_one.py C2
fi
echo done
