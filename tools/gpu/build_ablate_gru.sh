# Timing-ablation builds of the GRU update kernel (lib/libd2dhip_gabN.so, wrong gradients by design):
# D2D_GRU_ABLATE = 1 no weight-gradient GEMMs, 2 no dh MFMAs, 3 no history staging, 4 no BPTT recompute;
# cooperative path (record inputs): 5 exchange barriers and writes without the dW MFMAs, 6 no exchange;
# 7: the split step without its input products (W_ih fragments from L2).
# usage: bash tools/gpu/build_ablate_gru.sh [variants...]   (default 1 2 3 4)
# Run on the GPU box: python3 tools/gpu/ablate_gru.py
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
V="${*:-1 2 3 4}"
for n in $V; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc \
    -DD2D_GRU_ABLATE=$n $( [ "$n" = 7 ] && echo -DD2D_GRU_ABLATE_X=1 ) -c csrc/gru_kernels.hip -o build/abl/gru_kernels_$n.o &
done
wait
V="${*:-1 2 3 4}"
for n in $V; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_gab$n.so build/env_kernels.o \
    build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/abl/gru_kernels_$n.o build/abi.o
done
