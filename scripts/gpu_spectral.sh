cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_spectral_gpu.py tests/test_features_gpu.py -x -v -rf --timeout 120 --timeout-method thread > gpurun_out/spec_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/spec_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_spectral.py > gpurun_out/bench_spectral.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_spectral.log | tail -5
