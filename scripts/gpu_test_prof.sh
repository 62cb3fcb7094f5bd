# GPU tests, then bench.py + a rocprofv3 kernel trace (gpurun_out/prof).  Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh
