#!/bin/bash
# Does bench.py's driver-clock sampler (sysfs reads every 50 ms on a host
# thread) cost throughput?  Alternating on one box, 4 rounds.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for i in 1 2 3 4; do
  for s in 1 0; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --clock-sample $s > $OUT/sampler_$s_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.loads(open('$OUT/sampler_$s_$i.json').read().strip().splitlines()[-1]);print('sample=$s', d['value'], d['roofline'].get('clock_ghz_sysfs'))"
  done
done
