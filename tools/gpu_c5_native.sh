cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_lsp.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/cpp_gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/cpp_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_c5_native.py > gpurun_out/bench_c5_native.json 2> gpurun_out/bench_c5_native.err; rc=$?; cat gpurun_out/bench_c5_native.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_c5.py > gpurun_out/bench_c5_py.json 2> gpurun_out/bench_c5_py.err; cat gpurun_out/bench_c5_py.json
