# rocprofv3 runtime trace (HIP API + kernels) of a short bench run -> gpurun_out/rtrace (host issue vs GPU timing)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/rtrace
timeout -k 10 600 rocprofv3 --runtime-trace -d $R/gpurun_out/rtrace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-extras > $R/gpurun_out/rtrace.log 2>&1; rc=$?; echo "rtrace rc=$rc"
ls $R/gpurun_out/rtrace
exit $rc
