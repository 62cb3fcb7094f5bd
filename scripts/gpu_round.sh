# One GPU call: GPU test suite, smoke, bench (N=1, default: headline + extras + CPU baseline), rocprofv3
# kernel-trace of the bench command, PMC passes (FETCH_SIZE; WRITE_SIZE; MFMA busy — each its own run)
# -> gpurun_out/pmc_traffic.json.  Stops at the first failure.  SKIP_TESTS=1 skips the test suite.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
BENCH="python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras"
cd /tmp
rm -rf $R/gpurun_out/prof $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write $R/gpurun_out/pmc_mfma
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- $BENCH > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $BENCH --no-roofline > $R/gpurun_out/pmc_fetch.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- $BENCH --no-roofline > $R/gpurun_out/pmc_write.log 2>&1; rc=$?; echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_mfma -o run --output-format csv -- $BENCH --no-roofline > $R/gpurun_out/pmc_mfma.log 2>&1; rc=$?; echo "pmc mfma rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
python scripts/pmc_traffic.py gpurun_out/pmc_traffic.json gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof gpurun_out/pmc_mfma gpurun_out/bench.log > /dev/null; echo "pmc_traffic rc=$?"
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
