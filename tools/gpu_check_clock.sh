#!/bin/bash
# GPU check of bench.py's driver-clock sampler: the N = 1 line (issue bound at
# the sampled clock) and the 2-rank torchrun rehearsal (per-rank clocks).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_C2_clock.json 2> $OUT/bench_C2_clock.err || exit $?
python3 -c "import json;d=json.loads(open('$OUT/bench_C2_clock.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],r.get('clock_ghz_sysfs'),r['issue_bound'])"
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_rehearse2_clock.json 2> $OUT/bench_rehearse2_clock.err || exit $?
python3 -c "import json;d=json.loads(open('$OUT/bench_rehearse2_clock.json').read().strip().splitlines()[-1]);print(d['value'],d['result_ok'],d.get('clock_ghz_sysfs_per_rank'),d['config']['split'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_abi.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_multi.log 2>&1; tail -2 $OUT/gpu_multi.log
