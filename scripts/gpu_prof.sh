# bench.py (no CPU baseline) + rocprofv3 kernel trace of a short bench run -> gpurun_out/prof
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
