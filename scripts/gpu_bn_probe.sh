# Standalone BatchNorm backward pair at every bench shape: events (scripts/bench_bn.py) + per-kernel trace.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_bn.py > gpurun_out/bn.log 2>&1; rc=$?; cat gpurun_out/bn.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
rm -rf $R/gpurun_out/bnprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bnprof -o run --output-format csv -- python3 $R/scripts/bench_bn.py > $R/gpurun_out/bnprof.log 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
