# rocprofv3 kernel trace of scripts/bench_gemm.py (per-layer GEMM launches: kernel durations, grids)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/gtrace
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/gtrace -o run --output-format csv -- python3 $R/scripts/bench_gemm.py > $R/gpurun_out/gtrace.log 2>&1; rc=$?; echo "trace rc=$rc"
exit $rc
