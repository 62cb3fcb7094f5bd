set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_kmeans_gpu.py -x -q -k "edge_convs or wgrad or km or kmeans or bn_bwd" --timeout 120 --timeout-method thread > gpurun_out/t4_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t4_tests.log
[ $rc -eq 0 ] || exit $rc
HLMC_BENCH_ONLY=wgrad timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/wg_t4.log 2>&1; rc=$?; grep -E "wgrad|TOTAL" gpurun_out/wg_t4.log
timeout -k 10 300 python -u scripts/bench_bn.py > gpurun_out/bn_t4.log 2>&1; rc=$?; cat gpurun_out/bn_t4.log | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/kmeans_profile.py > gpurun_out/kmeans_profile.log 2>&1; rc=$?; echo "kmprof rc=$rc"; head -4 gpurun_out/kmeans_profile.log
cd /tmp
rm -rf $R/gpurun_out/bnprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bnprof -o run --output-format csv -- python3 $R/scripts/bench_bn.py > $R/gpurun_out/bnprof.log 2>&1; rc=$?; echo "bnprof rc=$rc"
