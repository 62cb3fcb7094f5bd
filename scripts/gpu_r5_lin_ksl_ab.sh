# Linear-layer split-K floor A/B (HLMC_LIN_MIN_KSL: minimum reduction length per split; 0 = 2 K-steps)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
HLMC_LIN_MIN_KSL=${TV:-1024} timeout -k 10 300 python -u -m pytest tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
for rep in 1 2 3; do
  for v in ${VALS:-0 512 1024 100000}; do
    l=$(HLMC_LIN_MIN_KSL=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras 2>&1 | grep '^{') || exit 1
    echo "ksl $v: $(echo "$l" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
