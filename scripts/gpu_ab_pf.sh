# register-path prefetch depth: GPU tests under HLMC_NT_PF=2, per-layer bench for 1 / 2, bench.py A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
HLMC_NT_PF=2 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; echo "tests(pf2) rc=$rc"; tail -1 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
for m in 1 2; do
  HLMC_NT_PF=$m timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm_pf$m.log 2>&1 || exit $?
done
for i in 1 2; do
  for m in 1 2; do
    HLMC_NT_PF=$m timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
    echo "pf=$m $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  done
done
