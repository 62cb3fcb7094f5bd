# Alternating bench.py A/B over a list of environment settings (KNOBS, ';'-separated; "-" = defaults), after the
# GPU tests in TESTS; then a kernel trace of the default build with its per-stream timeline.
#   KNOBS="-;HLMC_SIDE_STREAM=0" bash scripts/gpu_r3_knobs.sh [ROUNDS]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
N=${1:-3}
TESTS=${TESTS:-"tests/test_bench_parity_gpu.py tests/test_models_gpu.py"}
KNOBS=${KNOBS:-"-"}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/knob_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/knob_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
IFS=';' read -ra KS <<< "$KNOBS"
for i in $(seq 1 $N); do
  line="run $i:"
  j=0
  for k in "${KS[@]}"; do
    if [ "$k" = "-" ]; then envs=""; else envs="$k"; fi
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/knob_${j}_$i.log 2>&1 || exit 1
    line="$line  [$k] $(grep -o '"value": [0-9.]*' gpurun_out/knob_${j}_$i.log | cut -d' ' -f2)"
    j=$((j+1))
  done
  echo "$line"
done
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
cd $R
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
python scripts/step_gaps.py $f > gpurun_out/gaps.txt
grep -E "adam_pack" gpurun_out/crit.txt
