# Round-4 change check on one box: the GPU tests in TESTS, then an alternating A/B of the bench headline between the
# default and AB_ENV (an env knob of the same library), then bench_gemm per-layer timings.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ENV=${AB_ENV:-HLMC_SPLITK_FIX=0}
N=${ROUNDS:-3}
TESTS=${TESTS:-"tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_bench_parity_gpu.py tests/test_trainer_gpu.py"}
if [ -n "$TESTS" ] && [ "$TESTS" != "none" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ab_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab_def_$i.log 2>&1 || exit 1
  env $AB_ENV timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab_alt_$i.log 2>&1 || exit 1
  echo "run $i: default $(grep -o '"value": [0-9.]*' gpurun_out/ab_def_$i.log)  $AB_ENV $(grep -o '"value": [0-9.]*' gpurun_out/ab_alt_$i.log)"
done
if [ "${GEMM:-1}" = "1" ]; then
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit 1
env $AB_ENV timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_alt.log 2>&1 || exit 1
paste <(cut -c1-60 gpurun_out/bench_gemm.log) <(cut -c33-45 gpurun_out/bench_gemm_alt.log)
fi
