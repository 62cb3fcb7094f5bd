# Counter passes (kernel-trace only, one --pmc group per pass) for one op: bash scripts/pmc_op.sh TAG ARGS...
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; TAG=$1; shift
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_$TAG/t -o run --output-format csv -- python3 $R/scripts/op_probe.py "$@" > /dev/null 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc_$TAG/a -o run --output-format csv -- python3 $R/scripts/op_probe.py "$@" > /dev/null 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum -d $R/gpurun_out/pmc_$TAG/b -o run --output-format csv -- python3 $R/scripts/op_probe.py "$@" > /dev/null 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_$TAG/c -o run --output-format csv -- python3 $R/scripts/op_probe.py "$@" > /dev/null 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc_$TAG/d -o run --output-format csv -- python3 $R/scripts/op_probe.py "$@" > /dev/null 2>&1 || exit $?
echo "pmc $TAG done"
