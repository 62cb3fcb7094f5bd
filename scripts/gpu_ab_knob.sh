# Per-layer GEMM bench + bench.py A/B of one env knob, alternating on one box; GPU tests of the given files first.
#   bash scripts/gpu_ab_knob.sh VAR VALUE_A VALUE_B ROUNDS [TEST_FILES...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VAR=$1; A=$2; Bv=$3; N=$4; shift 4
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/knob_tests.log 2>&1; rc=$?
  tail -1 gpurun_out/knob_tests.log; [ $rc -eq 0 ] || exit $rc
fi
rm -f gpurun_out/sweep.log
for v in $A $Bv; do
  echo "== $VAR=$v" >> gpurun_out/sweep.log
  env $VAR=$v timeout -k 10 200 python scripts/bench_gemm.py >> gpurun_out/sweep.log 2>&1 || exit $?
done
bash scripts/gpu_ab_env.sh $VAR $A $Bv $N
