# A/B variants of the central critic's forward kernel (critic_kernels.hip), each linked with the product objects:
#   lib/libd2dhip_critpd2.so : D2D_CRITIC_PD=2, the operand prefetched one iteration ahead (two register sets)
#   lib/libd2dhip_critw8.so  : D2D_CRITIC_WAVES=8, 512-thread workgroups sharing each W1 image slice
#   lib/libd2dhip_critxl0.so : D2D_CRITIC_XLDS=0, the operand as fragment-shaped loads straight to registers
#   lib/libd2dhip_critwpd1.so: D2D_CRITIC_WPD=1, W1's image slices one iteration ahead (the XL path)
# (D2D_LIB_VARIANT=critpd2 / critw8 / critxl0 with D2D_ALLOW_ABLATION=1; tools/gpu/critic_probe.py)
# usage: bash tools/gpu/build_critic_variants.sh [variants...]   (default: all three)
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc"
VARS="${*:-pd2 w8 xl0}"
for v in $VARS; do
  case $v in
    pd2) D="-DD2D_CRITIC_PD=2 -DD2D_CRITIC_XLDS=0" ;;
    w8) D="-DD2D_CRITIC_WAVES=8 -DD2D_CRITIC_XLDS=0" ;;
    xl0) D="-DD2D_CRITIC_XLDS=0" ;;
    wpd1) D="-DD2D_CRITIC_WPD=1" ;;
  esac
  /opt/rocm/bin/hipcc $F $D -c csrc/critic_kernels.hip -o build/abl/critic_kernels_$v.o &
done
wait
for v in $VARS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_crit$v.so build/env_kernels.o \
    build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/gru_kernels.o \
    build/abl/critic_kernels_$v.o build/abi.o
done
