# Round-3 change check on one box: the GPU tests named in TESTS (default: ops, models, bench parity, e2e), then an
# alternating A/B of bench.py (headline only) between libhlmc_base.so (the previous build) and the current library,
# then a kernel trace of the current library with its per-stream timeline.
#   bash scripts/gpu_r3_ab_lib.sh [ROUNDS]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BASE=${BASE:-$R/hybrid-language-music-clustering-vae_amd/libhlmc_base.so}
N=${1:-3}
TESTS=${TESTS:-"tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_bench_parity_gpu.py tests/test_e2e_gpu.py"}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/lib_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/lib_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
for i in $(seq 1 $N); do
  HLMC_LIB=$BASE timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab_base_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  echo "run $i: base $(grep -o '"value": [0-9.]*' gpurun_out/ab_base_$i.log)  new $(grep -o '"value": [0-9.]*' gpurun_out/ab_new_$i.log)"
done
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-roofline > $R/gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
cd $R
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1); python scripts/step_critical.py $f 2 > gpurun_out/crit.txt; head -3 gpurun_out/crit.txt
python scripts/step_gaps.py $f > gpurun_out/gaps.txt
