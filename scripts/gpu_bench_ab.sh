# A/B of bench.py under env settings given as args "tag:VAR=val,VAR=val"; 2 alternating rounds; then models tests.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_trainer_gpu.py -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/models.log 2>&1; rc=$?; echo "models rc=$rc"; tail -2 gpurun_out/models.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/ab_$tag.log 2>&1; rc=$?
    echo "r$r $tag rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
