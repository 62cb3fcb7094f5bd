# Round 6 final, call 3: float4 split-K reduces (grouped TN, NT) -- op / parity / DP tests, per-layer conv GEMM times
# against abl/b1, step A/B, then the bench + profiles + PMC passes (gpu_round.sh with SKIP_TESTS=1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_dp_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fc_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fc_t.log
[ $rc -eq 0 ] || exit $rc
for n in main b1; do
  lib=abl/$n/libhlmc.so; [ $n = main ] && lib=hybrid-language-music-clustering-vae_amd/libhlmc.so
  echo "== $n" >> gpurun_out/fc_gemm.txt
  HLMC_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 180 python scripts/bench_gemm.py 2>&1 | grep -v "amdgpu.ids" >> gpurun_out/fc_gemm.txt || exit 2
done
bash scripts/gpu_ab.sh 3 "HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/b1/libhlmc.so" > gpurun_out/fc_ab.txt 2>&1 || exit 3
SKIP_TESTS=1 bash scripts/gpu_round.sh || exit $?
