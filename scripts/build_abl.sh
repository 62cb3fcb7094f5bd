# Build libhlmc variants that differ only in features.hip's ablation macro (HLMC_STFT_ABL=N) into
# hybrid-language-music-clustering-vae_amd/abl/libhlmc_abl<N>.so (measurement builds; not shipped)
set -e
cd "$(dirname "$0")/../hybrid-language-music-clustering-vae_amd/csrc"
mkdir -p ../abl ../build_abl
for N in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable \
    -ffp-contract=off -DHLMC_STFT_ABL=$N -c features.hip -o ../build_abl/features_$N.o
  objs=$(ls ../build/*.o | grep -v features.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../abl/libhlmc_abl$N.so $objs ../build_abl/features_$N.o
done
