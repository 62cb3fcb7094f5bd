# Round-4 targeted check: the tests named in TESTS (-k filter in KSEL), then the yardstick pass.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_dp_gpu.py"}
KSEL=${KSEL:-"halo or bf16_tracks or dp_two"}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s -k "$KSEL" --timeout 300 --timeout-method thread > gpurun_out/check_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error|halo|BN buffers|DP gradient" gpurun_out/check_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
[ "${YARD:-1}" = "1" ] && bash scripts/gpu_r4_yard.sh
