# Timing-ablation builds of libd2dhip (lib/libd2dhip_ablN.so); see tools/gpu/ablate_update.py.
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
for n in 1 2 3 4 5; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc \
    -DD2D_UPD_ABLATE=$n -c csrc/update_kernels.hip -o build/abl/update_kernels_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_abl$n.so build/env_kernels.o \
    build/gae_kernels.o build/policy_kernels.o build/abl/update_kernels_$n.o build/abi.o
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc \
  -DD2D_LOGITS_BF16=0 -c csrc/update_kernels.hip -o build/abl/update_kernels_lb.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_lf32.so build/env_kernels.o \
  build/gae_kernels.o build/policy_kernels.o build/abl/update_kernels_lb.o build/abi.o
