set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1}; do
  for rep in 1 2; do
    echo "variant $v: $(HLMC_LIB=build_ab/v$v/libhlmc.so timeout -k 10 120 python -u scripts/bench_mel.py 2>&1 | grep -v amdgpu.ids)"
  done
done
if [ -n "${TESTS:-}" ]; then
  HLMC_LIB=build_ab/v${TESTS}/libhlmc.so timeout -k 10 400 python -u -m pytest tests/test_features_gpu.py tests/test_bench_parity_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/stft_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/stft_tests.log
fi
