# round-3 full GPU pass: the whole -m gpu suite, smoke, the default bench (headline + extras + CPU baseline), an
# alternating A/B of one knob (AB_ENV, default HLMC_NT_TR=0) on the step, per-layer GEMM timings, a kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB_ENV=${AB_ENV:-HLMC_NT_TR=0}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/full_tests.log | tail -2
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --no-roofline --steps 30 > gpurun_out/ab_def_$i.log 2>&1 || exit 1
  env $AB_ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --no-roofline --steps 30 > gpurun_out/ab_alt_$i.log 2>&1 || exit 1
  echo "run $i: default $(python -c "import json; print(json.loads(open('gpurun_out/ab_def_$i.log').read().strip().splitlines()[-1])['value'])")  $AB_ENV $(python -c "import json; print(json.loads(open('gpurun_out/ab_alt_$i.log').read().strip().splitlines()[-1])['value'])")"
done
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit 1
tail -4 gpurun_out/bench_gemm.log
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
cd $R
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); python scripts/prof_summary.py $f 13 60 > gpurun_out/prof_summary.txt
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
