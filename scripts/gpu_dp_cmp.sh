cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in cur head; do
  envs=""; [ $lib = head ] && envs="HLMC_LIB=$GRAFT_REPO_ROOT/ab_libs/libhlmc_head.so"
  env $envs timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/dp_$lib.log 2>&1
  echo "== $lib rc=$?"; grep -E "rel L2|passed|failed" gpurun_out/dp_$lib.log | head -12
done
