set -o pipefail
mkdir -p gpurun_out
D=distributed_bitcoin_minter_amd
for v in pin cl pincl; do
  BTCMINER_LIB=$PWD/$D/libbtcminer_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/parity_$v.log 2>&1 || { echo "parity $v FAILED"; tail -20 gpurun_out/parity_$v.log; exit 1; }
  tail -1 gpurun_out/parity_$v.log
done
L="$D/libbtcminer.so $D/libbtcminer_pin.so $D/libbtcminer_cl.so $D/libbtcminer_pincl.so"
AB_REPS=5 timeout -k 10 600 python -u tools/ab_bench.py $L $L $L $L > gpurun_out/ab_pin_cluster.log 2>&1
echo "ab rc=$?"
