cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
for cfg in "1 --eager" "1 " "0 --eager" "0 "; do
  set -- $cfg
  HLMC_SIDE_STREAM=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 $2 > gpurun_out/ab.log 2>&1 || exit $?
  echo "side=$1 $2 $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
done; done
