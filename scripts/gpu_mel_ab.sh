cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_features_gpu.py tests/test_spectral_gpu.py tests/test_preprocess_gpu.py tests/test_e2e_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ft.log 2>&1; rc=$?; tail -1 gpurun_out/ft.log; grep -E "FAILED|Error" gpurun_out/ft.log | head -5; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc_base.so timeout -k 10 100 python scripts/bench_mel.py || exit 1
timeout -k 10 100 python scripts/bench_mel.py || exit 1
done
