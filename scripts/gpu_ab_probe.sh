# Probe overhead: bench default (live probe over the last HLMC_PROBE_STEPS timed steps) vs --no-roofline, alternating
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 5 3 off; do
    if [ $v = off ]; then a="--no-roofline"; else a=""; fi
    HLMC_PROBE_STEPS=${v/off/3} timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/ab.log 2>&1 || exit $?
    echo "probe=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"avg_us_per_launch": [0-9.]*' gpurun_out/ab.log)"
  done
done
