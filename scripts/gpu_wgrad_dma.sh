# Per-layer weight-gradient timing of the LDS-DMA TN kernel (HLMC_TN_DMA=1) under several grid targets / ring
# depths, beside the register-staged default.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" HLMC_BENCH_ONLY=wgrad timeout -k 10 200 python -u scripts/bench_gemm.py > gpurun_out/wgrad_$tag.log 2>&1 || exit $?
  echo "== $tag"; grep -E "wgrad|TOTAL" gpurun_out/wgrad_$tag.log | grep -v c1
}
run reg HLMC_X=1
for t in 128 256 512; do
  for ns in 4 8; do run dma_${t}_$ns HLMC_TN_DMA=1 HLMC_TN_DMA_BLOCKS=$t HLMC_TN_DMA_NS=$ns; done
done
