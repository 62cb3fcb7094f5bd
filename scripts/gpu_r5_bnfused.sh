# One-launch BatchNorm backward (bn_bwd_fused_kernel): its parity / repeatability tests, the standalone pair timing
# with and without it (HLMC_BN_FUSED=0: the two-pass form), then bench A/B rounds (headline only).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "bn_bwd" -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/bnf_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/bnf_tests.log
[ $rc -eq 0 ] || exit $rc
echo "fused:"; timeout -k 10 120 python scripts/bench_bn.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "two-pass:"; HLMC_BN_FUSED=0 timeout -k 10 120 python scripts/bench_bn.py 2>&1 | grep -v amdgpu.ids || exit 1
for rep in 1 2 3; do
  for v in ${LIMS:-8388608 0}; do
    l=$(HLMC_BN_FUSED=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras 2>&1 | grep '^{') || exit 1
    echo "lim $v: $(echo "$l" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
