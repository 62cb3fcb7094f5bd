# Per-layer weight-gradient timing (scripts/bench_gemm.py, wgrad family only) under several TN split-K grid targets.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in "$@"; do
  HLMC_BENCH_ONLY=wgrad HLMC_TN_BLOCKS=$t timeout -k 10 200 python -u scripts/bench_gemm.py > gpurun_out/wgrad_blocks_$t.log 2>&1 || exit $?
  echo "== TN_BLOCKS=$t"; grep -E "wgrad|TOTAL" gpurun_out/wgrad_blocks_$t.log | grep -v c1
done
