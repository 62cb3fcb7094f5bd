# Round 6: single-split weight gradients stored by their epilogue (no slab, no reduce launch) -- op / parity / DP /
# model tests, then step A/B against the committed library (abl/c1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_dp_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dir_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/dir_t.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh 3 "HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/c1/libhlmc.so" > gpurun_out/dir_ab.txt 2>&1 || exit 3
