set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-0}; do
  for rep in 1 2; do
    echo "variant $v: $(HLMC_LIB=build_ab/v$v/libhlmc.so timeout -k 10 120 python -u scripts/bench_mel.py 2>&1 | grep -v amdgpu.ids)"
  done
done
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; grep -oE "SQ_[A-Z_0-9]+" gpurun_out/avail.txt | sort -u | tr "\n" " " > gpurun_out/sq_counters.txt; echo
P=${PMC:-}
if [ -n "$P" ]; then
  HLMC_LIB=build_ab/v${PMCV:-0}/libhlmc.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/stft_pmc3 -o run --output-format csv -- python scripts/bench_mel.py > gpurun_out/stft_pmc3.log 2>&1; echo "pmc rc=$?"
fi
