set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "nr8:"; timeout -k 10 120 python scripts/bench_bn.py 2>&1 | grep -E "8x8|4x4" || exit 1
echo "nr4:"; HLMC_BN_FUSED_NR=4 timeout -k 10 120 python scripts/bench_bn.py 2>&1 | grep -E "8x8|4x4" || exit 1
for rep in 1 2 3; do
  for v in 8 4; do
    l=$(HLMC_BN_FUSED_NR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras 2>&1 | grep '^{') || exit 1
    echo "nr $v: $(echo "$l" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
