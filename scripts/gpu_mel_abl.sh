for n in 1 2 3; do HLMC_LIB=$GRAFT_REPO_ROOT/hybrid-language-music-clustering-vae_amd/abl/libhlmc_abl$n.so timeout -k 10 120 python scripts/bench_mel.py 256 2>&1 | grep mel_db | sed "s/^/abl$n /"; done
timeout -k 10 120 python scripts/bench_mel.py 256 2>&1 | grep mel_db | sed "s/^/main /"
