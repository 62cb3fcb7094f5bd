# Round 6 A/B of the working tree's library against a saved baseline (abl/$1/libhlmc.so): the TN/linear parity
# tests, per-layer weight-gradient times for both, then alternating bench rounds.  Usage: gpu_r6_cmp.sh BASE TAG
base=$1; tag=$2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 300 --timeout-method thread -k "wgrad or linear or train_step" > gpurun_out/${tag}_t.log 2>&1 || exit 1
for n in main $base; do
  lib=abl/$n/libhlmc.so; [ $n = main ] && lib=hybrid-language-music-clustering-vae_amd/libhlmc.so
  echo "== $n" >> gpurun_out/${tag}_gemm.txt
  HLMC_LIB=$GRAFT_REPO_ROOT/$lib HLMC_BENCH_ONLY=wgrad timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v "amdgpu.ids\|enc1\|dec5" >> gpurun_out/${tag}_gemm.txt || exit 2
done
bash scripts/gpu_ab.sh 3 "HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/$base/libhlmc.so" > gpurun_out/${tag}_ab.txt 2>&1 || exit 3
