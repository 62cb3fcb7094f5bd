# Per-layer weight-gradient timing (bench_gemm.py wgrad family) under env settings "tag:VAR=val,VAR=val".
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
  env $envs HLMC_BENCH_ONLY=wgrad timeout -k 10 200 python -u scripts/bench_gemm.py > gpurun_out/wgrad_$tag.log 2>&1 || exit $?
  echo "== $tag"; grep -E "wgrad|TOTAL" gpurun_out/wgrad_$tag.log | grep -v c1
done
