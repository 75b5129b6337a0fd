#!/bin/bash
# C4 on one GPU (2^40 nonces, one process) and the 8-slot one-process
# rehearsal of C4 with the range partitioner balancing (every slot on GPU 0):
# both answers must equal the full 2^40 CPU scan.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_C4_1gpu.json 2> $OUT/bench_C4_1gpu.err || exit $?
python3 -c "import json;d=json.loads(open('$OUT/bench_C4_1gpu.json').read().strip().splitlines()[-1]);print('C4 1gpu',d['value'],d['result_ok'],d['result'])"
timeout -k 10 300 python -u bench.py --config C4 --gpus 8 --rehearse-one-gpu --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_C4_rehearse8.json 2> $OUT/bench_C4_rehearse8.err || exit $?
python3 -c "import json;d=json.loads(open('$OUT/bench_C4_rehearse8.json').read().strip().splitlines()[-1]);print('C4 8-slot rehearsal',d['value'],d['result_ok'],d['result'],d['config']['split'])"
