# Round 6 final, call 5: bench + kernel trace + PMC traffic passes on the last library (tests ran in call 4's twin)
cd $GRAFT_REPO_ROOT && SKIP_TESTS=1 bash scripts/gpu_round.sh
