# Round-4: rehearse the self-launched N > 1 bench on the 1-GPU box (gloo, both ranks on cuda:0), plus the trainer tests.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/trainer_tests.log 2>&1; rc=$?
echo "trainer tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/trainer_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
HLMC_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --e2e-clips 2048 > gpurun_out/bench_n2.log 2> gpurun_out/bench_n2.err; rc=$?
echo "bench n2 rc=$rc"; tail -c 3000 gpurun_out/bench_n2.log; tail -5 gpurun_out/bench_n2.err
