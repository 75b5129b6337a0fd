#!/bin/bash
# Round-2 end-of-work GPU check in one gpurun call: smoke, the whole GPU
# suite, the default bench line, C5 at size through tools/bench_c5.py, an
# occupancy A/B, and a probe for a Go toolchain on the box.
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
(command -v go; command -v gccgo; go version) > $OUT/go_probe.log 2>&1; echo "go probe: $(head -c 200 $OUT/go_probe.log | tr '\n' ' ')"
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider -rs
step bench_C2 300 python -u bench.py --steps 20 --warmup 5
step bench_c5 400 python -u tools/bench_c5.py
if [ "${AB:-1}" = "1" ]; then
  for r in 1 2; do for b in 8 7 6; do export AB_BPC=$b; step ab_bpc_${b}_$r 200 python -u tools/ab_bench.py distributed_bitcoin_minter_amd/libbtcminer.so; done; done; unset AB_BPC
fi
echo done
