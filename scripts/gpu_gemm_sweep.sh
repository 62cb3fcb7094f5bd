# per-layer GEMM bench under pipeline / split-K / XCD-remap knobs (one process per setting, each under its own limit)
# usage: bash scripts/gpu_gemm_sweep.sh "CFG1" "CFG2" ...   (CFG = space-separated VAR=value list; "X=0" = defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/sweep.log
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/sweep.log
  env $cfg timeout -k 10 120 python scripts/bench_gemm.py >> gpurun_out/sweep.log 2>&1 || exit $?
done
echo done
