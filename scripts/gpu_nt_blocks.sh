# Per-layer NT (conv forward / data-gradient) timing (scripts/bench_gemm.py) under several split-K grid targets.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in "$@"; do
  for fam in conv subpixel; do
    HLMC_BENCH_ONLY=$fam HLMC_NT_BLOCKS=$t timeout -k 10 200 python -u scripts/bench_gemm.py > gpurun_out/nt_blocks_${fam}_$t.log 2>&1 || exit $?
    echo "== NT_BLOCKS=$t $fam"; grep -E "$fam|TOTAL" gpurun_out/nt_blocks_${fam}_$t.log | grep -v c1
  done
done
