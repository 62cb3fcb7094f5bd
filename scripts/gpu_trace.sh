# rocprofv3 kernel trace of a short bench run -> gpurun_out/prof_$1; critical-path summary
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-cur}; shift || true
cd /tmp
rm -rf $R/gpurun_out/prof_$tag
env "$@" timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $R/gpurun_out/prof_$tag.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
python scripts/step_critical.py $f 2 > gpurun_out/crit_$tag.txt; cat gpurun_out/crit_$tag.txt
