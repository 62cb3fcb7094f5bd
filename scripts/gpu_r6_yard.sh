# Round 6: deep-layer vendor yardstick (hipBLASLt dense / MIOpen) against the committed library
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_deep.py > gpurun_out/deep_yardstick_v2.txt 2>&1
