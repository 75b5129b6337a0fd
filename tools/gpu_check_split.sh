#!/bin/bash
# GPU check after the range partitioner: the whole GPU suite (parity of the
# rebuilt library, the weighted split and balance tests, the rehearsals),
# then the default bench line and a one-GPU 2-rank torchrun rehearsal with
# the split calibrated in the warmup.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_C2.json 2> $OUT/bench_C2.err || exit $?
cut -c1-300 $OUT/bench_C2.json
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --rehearse-one-gpu --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_rehearse2_split.json 2> $OUT/bench_rehearse2_split.err || exit $?
python3 -c "import json;d=json.loads(open('$OUT/bench_rehearse2_split.json').read().strip().splitlines()[-1]);print(d['value'],d['result_ok'],d['config']['split'])"
