# Env-kernel and GRU-policy ablation builds (lib/libd2dhip_<name>.so, D2D_LIB_VARIANT=<name> D2D_ALLOW_ABLATION=1,
# timed with tools/gpu/ablate_env.py): register budget (waves per SIMD), lane count of record-only
# comb steps, three-input xor in Philox.  Defaults: 7 waves, 256 lanes, xor3 (env_kernels.hip, common.h).
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
build() {  # name, extra flags
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
    $2 -c csrc/env_kernels.hip -o build/abl/env_kernels_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$1.so build/abl/env_kernels_$1.o \
    build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/gru_kernels.o build/abi.o
}
build envw6b512 "-DD2D_COMB_WAVES_PER_EU=6 -DD2D_COMB_REC_BLOCK=512" &
build envnox3 "-DD2D_PHILOX_XOR3=0" &
wait
# GRU policy step on eight-term splits (timing only)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
  -DD2D_GRU_SPLIT8=1 -c csrc/gru_kernels.hip -o build/abl/gru_kernels_s8.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_gru8.so build/env_kernels.o \
  build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/abl/gru_kernels_s8.o build/abi.o
