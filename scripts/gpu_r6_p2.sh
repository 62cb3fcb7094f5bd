# Round 6: weight-gradient TN loaders with buffer descriptors (power-of-two shapes) -- parity, per-layer, step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 300 --timeout-method thread -k "wgrad or linear or train_step" > gpurun_out/p2_t.log 2>&1 || exit 1
for n in main old; do
  lib=abl/$n/libhlmc.so; [ $n = main ] && lib=hybrid-language-music-clustering-vae_amd/libhlmc.so
  echo "== $n" >> gpurun_out/p2_gemm.txt
  HLMC_LIB=$GRAFT_REPO_ROOT/$lib HLMC_BENCH_ONLY=wgrad timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v "amdgpu.ids\|enc1\|dec5" >> gpurun_out/p2_gemm.txt || exit 2
done
bash scripts/gpu_ab.sh 3 "HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/old/libhlmc.so" > gpurun_out/p2_ab.txt 2>&1 || exit 3
