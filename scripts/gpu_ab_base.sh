# GPU tests (given files) with the current library, then bench.py A/B base library vs current, alternating.
#   bash scripts/gpu_ab_base.sh ROUNDS [TEST_FILES...]   (base = hybrid-language-music-clustering-vae_amd/libhlmc_base.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/libhlmc_base.so
N=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/base_tests.log 2>&1; rc=$?
  tail -1 gpurun_out/base_tests.log; grep -E "^FAILED|Error" gpurun_out/base_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 $N); do
  HLMC_LIB=$BASE timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
  echo "base $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/ab.log 2>&1 || exit $?
  echo "new  $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
done
