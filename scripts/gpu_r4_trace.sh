# rocprofv3 kernel trace of a short bench run (env from the caller) -> per-kernel stats of one step + step timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-cur}
cd /tmp
rm -rf $R/gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/tr_$TAG.log 2>&1; rc=$?; echo "trace rc=$rc"
cd $R
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
python scripts/step_critical.py $f 2 > gpurun_out/crit_$TAG.txt; head -30 gpurun_out/crit_$TAG.txt
python scripts/step_gaps.py $f > gpurun_out/gaps_$TAG.txt
