# Weight-gradient GEMM loader paths: op tests, bench_gemm wgrad timings (branch-free vector loads vs the
# per-element path, HLMC_TN_VEC=0), then the usual bench A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wv_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/wv_tests.log; exit 1; }
tail -1 gpurun_out/wv_tests.log
for k in "-" "HLMC_TN_VEC=0"; do
  envs=""; [ "$k" != "-" ] && envs="$k"
  env $envs HLMC_BENCH_ONLY=wgrad timeout -k 10 120 python scripts/bench_gemm.py > gpurun_out/wv_$k.log 2>&1 || { echo "bench_gemm failed"; exit 1; }
  echo "== $k"; grep -E "wgrad" gpurun_out/wv_$k.log
done
for i in 1 2 3; do
  line="run $i:"
  for k in "-" "HLMC_TN_VEC=0"; do
    envs=""; [ "$k" != "-" ] && envs="$k"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/wv_b.log 2>&1 || exit 1
    line="$line  [$k] $(grep -o '"value": [0-9.]*' gpurun_out/wv_b.log | cut -d' ' -f2)"
  done
  echo "$line"
done
