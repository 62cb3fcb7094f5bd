# Alternating A/B of environment settings on bench.py (one box, fixed order per round):
#   bash scripts/gpu_ab.sh ROUNDS "ENV_A" "ENV_B" ...   (each ENV_x: space-separated VAR=value pairs, or "-")
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
N=$1; shift
for i in $(seq 1 $N); do
  for cfg in "$@"; do
    [ "$cfg" = "-" ] && envs="" || envs="$cfg"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
    echo "[$cfg] $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
