# Halo-kernel variants: op tests, then the conv_s2 / subpixel op timings of scripts/bench_gemm.py for the in-tree
# library and each ab_libs/libhlmc_<name>.so given as arguments, then an alternating bench.py A/B over the same.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/halo_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
for v in cur "$@"; do
  lib=""; [ $v != cur ] && lib="HLMC_LIB=$GRAFT_REPO_ROOT/ab_libs/libhlmc_$v.so"
  for f in conv subpixel; do
    env $lib HLMC_BENCH_ONLY=$f timeout -k 10 120 python scripts/bench_gemm.py > gpurun_out/halo_${v}_$f.log 2>&1 || { echo "$v $f failed"; tail -5 gpurun_out/halo_${v}_$f.log; exit 1; }
  done
  echo "== $v"; grep -h -E "conv_s2|subpixel" gpurun_out/halo_${v}_conv.log gpurun_out/halo_${v}_subpixel.log | grep -E " (64|32|16)x"
done
for i in 1 2 3; do
  line="run $i:"
  for v in cur "$@"; do
    lib=""; [ $v != cur ] && lib="HLMC_LIB=$GRAFT_REPO_ROOT/ab_libs/libhlmc_$v.so"
    env $lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-extras --steps 40 > gpurun_out/halo_b_$v.log 2>&1 || exit 1
    line="$line  [$v] $(grep -o '"value": [0-9.]*' gpurun_out/halo_b_$v.log | cut -d' ' -f2)"
  done
  echo "$line"
done
