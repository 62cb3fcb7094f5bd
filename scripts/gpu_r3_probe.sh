# round-3 probe: the new / changed GPU tests with their printed errors (no -x: collect every number), then the bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bench_parity_gpu.py tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py tests/test_dp_gpu.py tests/test_kmeans_gpu.py tests/test_trainer_gpu.py -q -s -rf --timeout 300 --timeout-method thread > gpurun_out/probe_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/probe_tests.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
