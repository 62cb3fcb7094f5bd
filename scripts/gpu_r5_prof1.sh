# Round 5: K-Means host/device breakdown; weight-gradient kernel vs reduce split (rocprofv3 kernel trace) and
# stall counters of the TN kernel.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/kmeans_profile.py > gpurun_out/kmeans_profile.log 2>&1; rc=$?; echo "kmprof rc=$rc"; head -12 gpurun_out/kmeans_profile.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
rm -rf $R/gpurun_out/wgprof $R/gpurun_out/wgpmc
HLMC_BENCH_ONLY=wgrad timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wgprof -o run --output-format csv -- python3 $R/scripts/bench_gemm.py > $R/gpurun_out/wgprof.log 2>&1; rc=$?; echo "wgprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
HLMC_BENCH_ONLY=wgrad timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/wgpmc -o run --output-format csv -- python3 $R/scripts/bench_gemm.py > $R/gpurun_out/wgpmc.log 2>&1; rc=$?; echo "wgpmc rc=$rc"
