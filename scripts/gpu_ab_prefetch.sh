# GPU tests, then A/B on one box: base library vs current (edge kernels), and mel prefetch on/off
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh 1 || exit $?
for i in 1 2; do
  for a in "--no-prefetch" ""; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 $a > gpurun_out/ab.log 2>&1 || exit $?
    echo "[$a] $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
