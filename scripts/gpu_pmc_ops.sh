# PMC counter passes for representative conv GEMM launches (scripts/pmc_op.sh): wgrad 32-ch and 128-ch,
# sub-pixel 64->32, conv 32->64
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 bash scripts/pmc_op.sh wg1 wgrad 256 32 32 64 32 > gpurun_out/pmc_wg1.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/pmc_op.sh wg4 wgrad 256 8 8 256 128 > gpurun_out/pmc_wg4.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/pmc_op.sh sp4 subpixel 256 32 32 64 32 > gpurun_out/pmc_sp4.log 2>&1 || exit $?
timeout -k 10 400 bash scripts/pmc_op.sh cv1 conv 256 64 64 32 64 > gpurun_out/pmc_cv1.log 2>&1 || exit $?
echo done
