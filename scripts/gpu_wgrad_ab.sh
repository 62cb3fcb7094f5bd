# wgrad DMA kernel: op tests, per-layer sweep (register-staged vs LDS-DMA ring depth / grid target), bench A/B.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -rf -k "wgrad or linear" > gpurun_out/ops.log 2>&1; rc=$?; echo "ops rc=$rc"; tail -2 gpurun_out/ops.log
[ $rc -eq 0 ] || exit $rc
run() {  # tag env...
  tag=$1; shift
  env "$@" HLMC_BENCH_ONLY=wgrad timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/wg_$tag.log 2>&1; rc=$?
  echo "== $tag rc=$rc: $(grep -E 'wgrad wgrad' gpurun_out/wg_$tag.log | awk '{printf "%s ", $5}') | $(grep TOTAL gpurun_out/wg_$tag.log)"
  return $rc
}
run reg HLMC_TN_DMA=0 || exit 1
for ns in 4 8; do for tb in 256 512 1024; do run ns${ns}_tb$tb HLMC_TN_DMA_NS=$ns HLMC_TN_DMA_BLOCKS=$tb || exit 1; done; done
