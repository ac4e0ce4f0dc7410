# Precision variants of the GRU update kernel (lib/libd2dhip_<v>.so; A/B and diagnosis only):
#   gdw0: weight-gradient GEMMs on fp32 MFMAs (D2D_GRU_DW_BF16=0); gdh0: BPTT dh on fp32 MFMAs (D2D_GRU_DH_BF16=0)
# usage: bash tools/gpu/build_gru_precision.sh
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc"
/opt/rocm/bin/hipcc $F -DD2D_GRU_DW_BF16=0 -c csrc/gru_kernels.hip -o build/abl/gru_kernels_gdw0.o &
/opt/rocm/bin/hipcc $F -DD2D_GRU_DH_BF16=0 -c csrc/gru_kernels.hip -o build/abl/gru_kernels_gdh0.o &
wait
for v in gdw0 gdh0; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$v.so build/env_kernels.o \
    build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/abl/gru_kernels_$v.o build/abi.o
done
