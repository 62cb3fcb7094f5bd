# One GPU call: GPU test suite, smoke, bench (N=1), rocprofv3 kernel-trace of the bench command, PMC
# passes (FETCH_SIZE, WRITE_SIZE; each its own run) -> gpurun_out/pmc_traffic.json.  Stops at the first failure.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmc_fetch.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmc_write.log 2>&1; rc=$?; echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
python scripts/pmc_traffic.py gpurun_out/pmc_traffic.json gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/prof > /dev/null; echo "pmc_traffic rc=$?"
