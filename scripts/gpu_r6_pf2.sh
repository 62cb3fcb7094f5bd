# Round 6: TN loads two K-steps ahead (PF2) and/or MFMA accumulators in VGPRs (-amdgpu-mfma-vgpr-form) -- parity of
# the candidate, per-layer conv GEMM times of every variant, then step A/B against the committed library (abl/b1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
HLMC_LIB=$GRAFT_REPO_ROOT/abl/v1/libhlmc.so timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pf2_t.log 2>&1 || exit 1
for n in b1 v1 v2 v3; do
  echo "== $n" >> gpurun_out/pf2_gemm.txt
  HLMC_LIB=$GRAFT_REPO_ROOT/abl/$n/libhlmc.so timeout -k 10 180 python scripts/bench_gemm.py 2>&1 | grep -v "amdgpu.ids" >> gpurun_out/pf2_gemm.txt || exit 2
done
bash scripts/gpu_ab.sh 2 "HLMC_LIB=$GRAFT_REPO_ROOT/abl/v1/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/b1/libhlmc.so" > gpurun_out/pf2_ab1.txt 2>&1 || exit 3
bash scripts/gpu_ab.sh 2 "HLMC_LIB=$GRAFT_REPO_ROOT/abl/v3/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/b1/libhlmc.so" > gpurun_out/pf2_ab3.txt 2>&1 || exit 4
