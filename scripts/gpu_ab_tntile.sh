# Per-layer weight-gradient timing under each HLMC_TN_TILE policy, then bench.py A/B of the two policies
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for m in 1 2; do
  HLMC_TN_TILE=$m timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_tn$m.log 2>&1 || exit $?
done
for i in 1 2; do
  for m in 1 2; do
    HLMC_TN_TILE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
    echo "tn=$m $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
