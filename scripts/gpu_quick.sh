# Quick GPU iteration: GPU tests, per-layer GEMM bench, bench.py (no CPU baseline). Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; rc=$?; echo "bench_gemm rc=$rc"; tail -1 gpurun_out/bench_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
