#!/bin/bash
# PMC passes for C3 (one block per pass) on the current build.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_C3_fetch -o f --output-format csv -- python3 tools/prof_one.py C3 2 > $OUT/pmc_C3_fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_C3_write -o w --output-format csv -- python3 tools/prof_one.py C3 2 > $OUT/pmc_C3_write.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d $OUT/pmc_C3_sq -o s --output-format csv -- python3 tools/prof_one.py C3 2 > $OUT/pmc_C3_sq.log 2>&1 || exit $?
echo pmc C3 done
