# round-3 A/B probe: re-run the fixed tests, then HLMC_NT_TR=1 vs 0 (transposed-accumulator epilogue) per layer and
# on the whole step (alternating), then a kernel trace of the default build.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_bench_parity_gpu.py tests/test_dp_gpu.py "tests/test_models_gpu.py::test_eval_mode_matches_fixture_chain" -q -s -rf --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/ab_tests.log | tail -2
[ $rc -le 1 ] || exit $rc
for tr in 1 0; do HLMC_NT_TR=$tr timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_tr$tr.log 2>&1 || exit 1; done
echo "bench_gemm done"
for i in 1 2; do for tr in 1 0; do
  HLMC_NT_TR=$tr timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --no-roofline --steps 30 > gpurun_out/ab_tr${tr}_$i.log 2>&1 || exit 1
  echo "TR=$tr run $i: $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_tr${tr}_$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done; done
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
cd $R
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); python scripts/prof_summary.py $f 13 60 > gpurun_out/prof_summary.txt
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
