# Alternating A/B of the bench headline over several env settings (KNOBS, ';'-separated; "-" = default), ROUNDS
# rounds, then optional extra commands (EXTRA).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
N=${ROUNDS:-3}
IFS=';' read -ra KS <<< "${KNOBS:--}"
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/knob_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/knob_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 $N); do
  line="run $i:"
  for k in "${KS[@]}"; do
    if [ "$k" = "-" ]; then e=""; else e="$k"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/knob.log 2>&1 || { echo "bench failed for $k"; tail -5 gpurun_out/knob.log; exit 1; }
    line="$line  [$k] $(grep -o '"value": [0-9.]*' gpurun_out/knob.log | cut -d' ' -f2)"
  done
  echo "$line"
done
if [ -n "$EXTRA" ]; then bash -c "$EXTRA"; fi
