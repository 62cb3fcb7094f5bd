# Host enqueue time vs GPU time of the bench step, then a runtime trace (HIP API + kernels) of a short bench run.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/host_overhead.py > gpurun_out/host_overhead.log 2>&1; rc=$?; echo "host rc=$rc"; cat gpurun_out/host_overhead.log | grep steps
[ $rc -eq 0 ] || exit $rc
cd /tmp
rm -rf $R/gpurun_out/rtrace
timeout -k 10 600 rocprofv3 --runtime-trace -d $R/gpurun_out/rtrace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-extras > $R/gpurun_out/rtrace.log 2>&1; rc=$?; echo "rtrace rc=$rc"
find $R/gpurun_out/rtrace -name "*.csv" | head
