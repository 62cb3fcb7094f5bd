# One fp32 train step (scripts/debug_bn_in.py) with the in-tree library and with ab_libs/libhlmc_$1.so; prints every
# tensor that differs at all (DBG_THR=0).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DBG_DTYPE=fp32 timeout -k 10 120 python scripts/debug_bn_in.py run cur > gpurun_out/dbg_cur.log 2>&1 || { tail -5 gpurun_out/dbg_cur.log; exit 1; }
HLMC_LIB=$GRAFT_REPO_ROOT/ab_libs/libhlmc_$1.so DBG_DTYPE=fp32 timeout -k 10 120 python scripts/debug_bn_in.py run old > gpurun_out/dbg_old.log 2>&1 || { tail -5 gpurun_out/dbg_old.log; exit 1; }
DBG_THR=0 python scripts/debug_bn_in.py cmp cur old | head -40
