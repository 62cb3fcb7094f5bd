set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_bn.py > gpurun_out/bn_t5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bn_t5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/kmeans_profile.py > gpurun_out/kmeans_profile.log 2>&1; rc=$?; echo "kmprof rc=$rc"; head -4 gpurun_out/kmeans_profile.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; python -c "
import json; l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')][-1]; d=json.loads(l); print('HEADLINE', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
