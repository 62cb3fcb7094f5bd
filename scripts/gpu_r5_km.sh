# Round 5: K-Means (restart-batched) GPU tests + benchmark, then the rest of the GPU suite.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py tests/test_e2e_gpu.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/km_tests.log 2>&1; rc=$?; echo "km tests rc=$rc"; tail -4 gpurun_out/km_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_kmeans.py > gpurun_out/bench_kmeans.log 2>&1; rc=$?; echo "bench_kmeans rc=$rc"; cat gpurun_out/bench_kmeans.log | grep case
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log
