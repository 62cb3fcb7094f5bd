# Alternating A/B of several env configurations of bench.py on one box:
#   bash scripts/gpu_ab_cfgs.sh ROUNDS "CFG1" "CFG2" ...   (CFG = space-separated VAR=value list; "X=0" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
N=$1; shift
for i in $(seq 1 $N); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
    echo "[$cfg] $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
