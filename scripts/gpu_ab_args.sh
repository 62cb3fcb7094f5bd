# A/B of two bench.py argument sets, alternating on one box:  bash scripts/gpu_ab_args.sh "ARGS_A" "ARGS_B" [ROUNDS]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
A=$1; Bv=$2; N=${3:-3}
for i in $(seq 1 $N); do
  for v in "$A" "$Bv"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $v > gpurun_out/ab.log 2>&1 || exit $?
    echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
