#!/bin/bash
# The GPU checks of a round, in one gpurun call; each phase named on the
# command line runs under its own time limit, and the script stops at the
# first phase that faults, aborts or times out (gpurun rules).
#   tools/gpu_round.sh smoke tests bench
#   phases: smoke | tests | tests_multi | bench | bench_c3 | bench_c4 | rehearse | prof | pmc | parity
# Logs and profiles land in gpurun_out/$TAG (TAG defaults to r03).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  # 1 = test failures / a wrong answer: reported, the next phase still runs;
  # anything else (fault, abort, timeout, signal) ends the call here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
PYTEST="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rs"
for phase in "$@"; do
  case $phase in
    smoke) step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step gpu_tests 1000 $PYTEST tests -m gpu -v ;;
    tests_multi) step gpu_tests_multi 600 $PYTEST tests/test_gpu_multi.py -m gpu -v ;;
    bench) step bench_C2 300 python -u bench.py --steps 20 --warmup 5 ;;
    bench_c3) step bench_C3 300 python -u bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c4) step bench_C4 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    rehearse)
      step rehearse2_oneproc 300 python -u bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline --rehearse-one-gpu
      step rehearse2_mask 300 env HIP_VISIBLE_DEVICES=0 python -u -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 ;;
    prof)
      # 1-stream kernel trace of the C2 bench (the dominant launch alone on its stream)
      step prof_C2 300 env BTCMINER_STREAMS=1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_C2" -o run \
        -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc)
      step pmc_sq 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/pmc_sq" -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
      step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
      step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    parity) step parity_campaign 600 python -u tools/parity_campaign.py 3000 303 ;;
    *) echo "unknown phase $phase"; exit 2 ;;
  esac
done
echo "done ($(date +%T))"
