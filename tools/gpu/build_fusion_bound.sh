# Timing variant for tools/gpu/fusion_bound.py: the policy kernel without its obs / record reads
# (lib/libd2dhip_noread.so; D2D_POLICY_ABLATE_NOREAD, wrong actions -- timing only)
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
  -DD2D_POLICY_ABLATE_NOREAD=1 -c csrc/policy_kernels.hip -o build/abl/policy_kernels_noread.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_noread.so build/env_kernels.o \
  build/gae_kernels.o build/abl/policy_kernels_noread.o build/update_kernels.o build/gru_kernels.o \
  build/critic_kernels.o build/abi.o
