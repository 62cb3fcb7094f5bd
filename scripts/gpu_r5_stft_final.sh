# STFT kernel evidence for profiles/r05: rocprofv3 kernel stats of scripts/bench_mel.py and two PMC passes.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/stft_final
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stft_final/trace -o run --output-format csv -- python3 $R/scripts/bench_mel.py > $R/gpurun_out/stft_final_trace.log 2>&1; echo "trace rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $R/gpurun_out/stft_final/pmc1 -o run --output-format csv -- python3 $R/scripts/bench_mel.py > $R/gpurun_out/stft_final_pmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS -d $R/gpurun_out/stft_final/pmc2 -o run --output-format csv -- python3 $R/scripts/bench_mel.py > $R/gpurun_out/stft_final_pmc2.log 2>&1; echo "pmc2 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/stft_final/fetch -o run --output-format csv -- python3 $R/scripts/bench_mel.py > $R/gpurun_out/stft_final_fetch.log 2>&1; echo "fetch rc=$?"
