# A/B of two library builds on one box: per-layer GEMM/edge bench and bench.py with HLMC_LIB=base vs current.
#   bash scripts/gpu_ab_lib.sh [ROUNDS]   (base = hybrid-language-music-clustering-vae_amd/libhlmc_base.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc_base.so
N=${1:-2}
HLMC_LIB=$BASE timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_base.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit $?
for i in $(seq 1 $N); do
  HLMC_LIB=$BASE timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
  echo "base $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
  echo "new  $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
done
