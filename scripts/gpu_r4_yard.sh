# Round-4 yardstick pass: deep-layer vendor comparison (bench_deep.py), per-layer GEMM timings, headline bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_deep.py > gpurun_out/deep.log 2>&1; rc=$?; echo "deep rc=$rc"; cat gpurun_out/deep.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; rc=$?; echo "bench_gemm rc=$rc"; tail -3 gpurun_out/bench_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
