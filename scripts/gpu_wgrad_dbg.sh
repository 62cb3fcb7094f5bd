set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -rf -k "wgrad or linear" > gpurun_out/ops.log 2>&1; rc=$?; echo "ops rc=$rc"; tail -2 gpurun_out/ops.log
[ $rc -eq 0 ] || exit $rc
run() {
  tag=$1; shift
  env "$@" HLMC_BENCH_ONLY=wgrad timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/wg_$tag.log 2>&1; rc=$?
  echo "== $tag rc=$rc: $(grep -E 'wgrad wgrad' gpurun_out/wg_$tag.log | awk '{printf "%s ", $5}') | $(grep TOTAL gpurun_out/wg_$tag.log)"
  return $rc
}
run reg HLMC_TN_DMA=0 || exit 1
run reg1024 HLMC_TN_DMA=0 HLMC_TN_BLOCKS=1024 || exit 1
run reg256 HLMC_TN_DMA=0 HLMC_TN_BLOCKS=256 || exit 1
run full HLMC_TN_DMA_NS=4 || exit 1
run full512 HLMC_TN_DMA_NS=4 HLMC_TN_DMA_BLOCKS=512 || exit 1
run nocompute HLMC_TN_DMA_NS=4 HLMC_TN_DMA_DBG=1 || exit 1
run noissue HLMC_TN_DMA_NS=4 HLMC_TN_DMA_DBG=2 || exit 1
run nothing HLMC_TN_DMA_NS=4 HLMC_TN_DMA_DBG=3 || exit 1
