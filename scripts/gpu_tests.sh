cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -rf > gpurun_out/ops.log 2>&1; rc=$?; echo "ops rc=$rc"; tail -3 gpurun_out/ops.log
if [ $rc -le 1 ]; then
  timeout -k 10 900 python -m pytest tests/test_models_gpu.py tests/test_features_gpu.py tests/test_kmeans_gpu.py -q -rf > gpurun_out/rest.log 2>&1; rc2=$?; echo "rest rc=$rc2"; tail -3 gpurun_out/rest.log
fi
