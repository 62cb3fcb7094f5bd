# Round 6 final, call 2: the weight-gradient op tests (the library changed after call 1), per-layer weight-gradient
# times against abl/b1, then bench (default: headline + extras + CPU baseline), rocprofv3 kernel trace, PMC traffic
# passes (gpu_round.sh with SKIP_TESTS=1), and counter passes over the deep forward conv / sub-pixel ops
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fb_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fb_t.log
[ $rc -eq 0 ] || exit $rc
for n in main b1; do
  lib=abl/$n/libhlmc.so; [ $n = main ] && lib=hybrid-language-music-clustering-vae_amd/libhlmc.so
  echo "== $n" >> gpurun_out/fb_gemm.txt
  HLMC_LIB=$GRAFT_REPO_ROOT/$lib HLMC_BENCH_ONLY=wgrad timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v "amdgpu.ids" >> gpurun_out/fb_gemm.txt || exit 2
done
SKIP_TESTS=1 bash scripts/gpu_round.sh || exit $?
bash scripts/pmc_op.sh conv5 conv 256 8 8 256 512 && bash scripts/pmc_op.sh sp5 subpixel 256 4 4 512 256
