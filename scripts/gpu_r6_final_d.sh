# Round 6 final, call 4 (library after the single-split direct store): the whole of gpu_round.sh -- GPU test suite,
# smoke, bench (default), rocprofv3 kernel trace, PMC traffic passes
cd $GRAFT_REPO_ROOT && bash scripts/gpu_round.sh
