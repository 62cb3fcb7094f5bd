# A/B of the XCD-aware block order per GEMM family: per-layer GEMM bench + bench.py with HLMC_XCD_REMAP=0 / 31
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for m in 0 31; do
  HLMC_XCD_REMAP=$m timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_rm$m.log 2>&1 || exit $?
  HLMC_XCD_REMAP=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_rm$m.log 2>&1 || exit $?
done
echo ok
