cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "wgrad or linear" > gpurun_out/tg2_t.log 2>&1 || exit 1
bash scripts/gpu_ab.sh 3 "HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc.so" "HLMC_LIB=$GRAFT_REPO_ROOT/abl/c4/libhlmc.so" > gpurun_out/tg2_ab.txt 2>&1 || exit 3
