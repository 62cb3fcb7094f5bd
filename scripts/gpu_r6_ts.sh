cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
HLMC_LIB=$GRAFT_REPO_ROOT/abl/ts/libhlmc.so timeout -k 10 120 python scripts/tn_ts.py > gpurun_out/tn_ts.txt 2>&1
