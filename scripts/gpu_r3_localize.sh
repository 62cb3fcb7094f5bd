cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in "-" "HLMC_BN_IN=0" "HLMC_BN_MOM_EPI=0" "HLMC_BN_IN=0 HLMC_BN_MOM_EPI=0"; do
  if [ "$k" = "-" ]; then e=""; else e="$k"; fi
  env $e timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k "bf16_mode or test_model_step" -x -q --timeout 200 --timeout-method thread > gpurun_out/loc.log 2>&1; rc=$?
  echo "[$k] rc=$rc $(grep -E 'passed|failed' gpurun_out/loc.log | tail -1)"
  [ $rc -le 1 ] || exit $rc
done
