set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "edge_convs" --timeout 120 --timeout-method thread > gpurun_out/edge_tests.log 2>&1; rc=$?; echo "edge tests rc=$rc"; tail -3 gpurun_out/edge_tests.log
[ $rc -eq 0 ] || exit $rc
HLMC_BENCH_ONLY=wgrad timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/wg_c1.log 2>&1; rc=$?; grep "wgrad_c1" gpurun_out/wg_c1.log
bash scripts/gpu_r5_prof2.sh
