# r03 A/B of the update kernels' tiles-per-wave cap (lib/libd2dhip_<v>.so; timing with
# tools/gpu/ablate_update.py <v> ...): w64 / w128: at most 64 / 128 tiles per wave (G = 50 / 25
# workgroups per agent at 2,048 envs x 200 slots; the default 256 leaves G = 16 there).
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc"
OTHER="build/env_kernels.o build/gae_kernels.o build/policy_kernels.o build/gru_kernels.o build/abi.o"
build() {  # name, source, extra flags
  /opt/rocm/bin/hipcc $F $3 -c $2 -o build/abl/upd_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$1.so $OTHER build/abl/upd_$1.o
}
build w64 csrc/update_kernels.hip "-DD2D_UPD_MAX_WAVE_TILES=64" &
build w128 csrc/update_kernels.hip "-DD2D_UPD_MAX_WAVE_TILES=128" &
wait
