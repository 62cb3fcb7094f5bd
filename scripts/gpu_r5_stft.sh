set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_features_gpu.py tests/test_bench_parity_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/stft_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/stft_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/bench_mel.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/stftprof -o run --output-format csv -- python scripts/bench_mel.py > gpurun_out/stftprof.log 2>&1; echo "prof rc=$?"
python -c "
import csv,glob
f=glob.glob('gpurun_out/stftprof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:4]: print(r['Name'][:60], r['Calls'], r['AverageNs'])"

