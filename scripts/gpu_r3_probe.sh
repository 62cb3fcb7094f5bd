# round-3 probe: the new / changed GPU tests with their printed errors (no -x: collect every number), the bench, and a
# rocprofv3 kernel-trace of a short bench (per-kernel times + the per-step critical path)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py tests/test_dp_gpu.py tests/test_kmeans_gpu.py tests/test_trainer_gpu.py -q -s -rf --timeout 300 --timeout-method thread > gpurun_out/probe_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/probe_tests.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
cd $R
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); python scripts/prof_summary.py $f 13 60 > gpurun_out/prof_summary.txt
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
