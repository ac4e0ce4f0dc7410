# A/B variant of the central critic's forward kernel with the round-5 first version's operand prefetch (one
# iteration ahead, two register sets: D2D_CRITIC_PD=2) -> lib/libd2dhip_critpd2.so (D2D_LIB_VARIANT=critpd2)
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
  -DD2D_CRITIC_PD=2 -c csrc/critic_kernels.hip -o build/abl/critic_kernels_pd2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_critpd2.so build/env_kernels.o \
  build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/gru_kernels.o \
  build/abl/critic_kernels_pd2.o build/abi.o
