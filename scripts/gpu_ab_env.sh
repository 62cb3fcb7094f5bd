# A/B of an environment toggle on bench.py, alternating on one box:  bash scripts/gpu_ab_env.sh VAR VALUE_A VALUE_B [ROUNDS]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VAR=$1; A=$2; Bv=$3; N=${4:-3}
for i in $(seq 1 $N); do
  for v in $A $Bv; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
    echo "$VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
