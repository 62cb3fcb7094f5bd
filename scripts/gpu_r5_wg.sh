# Round 5: LDS-DMA weight-gradient kernel: op tests, per-layer A/B of HLMC_TN_GLDS modes, then K-Means + full suite.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q -rf -k "wgrad" --timeout 300 --timeout-method thread > gpurun_out/wg_tests.log 2>&1; rc=$?; echo "wgrad tests rc=$rc"; tail -3 gpurun_out/wg_tests.log
[ $rc -eq 0 ] || exit $rc
for m in 0 1 2 3; do
  HLMC_TN_GLDS=$m HLMC_BENCH_ONLY=wgrad timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/wg_mode$m.log 2>&1; rc=$?; echo "mode $m rc=$rc"; grep -E "wgrad|TOTAL" gpurun_out/wg_mode$m.log
  [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r5_km.sh
