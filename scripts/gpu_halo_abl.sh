# Halo-kernel ablation (measurement only): the conv_s2 / subpixel op timings of scripts/bench_gemm.py for the
# in-tree library and ab_libs/libhlmc_abl{1,2,3}.so (built with -DHLMC_HALO_ABL=1 no MFMA, 2 no epilogue stores,
# 3 no global input loads).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 0 1 2 3; do
  lib=""; [ $v -ne 0 ] && lib="HLMC_LIB=$GRAFT_REPO_ROOT/ab_libs/libhlmc_abl$v.so"
  for f in conv subpixel; do
    env $lib HLMC_BENCH_ONLY=$f timeout -k 10 120 python scripts/bench_gemm.py > gpurun_out/abl_${v}_$f.log 2>&1 || { echo "abl $v $f failed"; tail -5 gpurun_out/abl_${v}_$f.log; exit 1; }
  done
  echo "== abl $v"; grep -h -E "conv_s2|subpixel" gpurun_out/abl_${v}_conv.log gpurun_out/abl_${v}_subpixel.log | grep -E " (64|32)x"
done
