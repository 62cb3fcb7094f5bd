# PMC counters for the mel stage micro-benchmark (separate passes; kernel-trace only)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -m pytest $R/tests/test_features_gpu.py -q -x 2>&1 | tail -3 && timeout -k 10 120 python3 $R/scripts/bench_mel.py || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/melpmc1 -o run --output-format csv -- python3 $R/scripts/bench_mel.py > /dev/null 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F32 SQ_BUSY_CYCLES -d $R/gpurun_out/melpmc2 -o run --output-format csv -- python3 $R/scripts/bench_mel.py > /dev/null 2>&1 || exit $?
ls $R/gpurun_out/melpmc1 $R/gpurun_out/melpmc2
