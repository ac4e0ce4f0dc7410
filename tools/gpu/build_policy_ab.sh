# A/B builds of the behaviour-policy kernel (lib/libd2dhip_<v>.so; timing only, selected with
# D2D_LIB_VARIANT=<v> D2D_ALLOW_ABLATION=1): pl2f: actor layer 2 on fp32 MFMA (D2D_POLICY_L2_F32=1);
# usage: bash tools/gpu/build_policy_ab.sh
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc"
# pl2f2: the same on two accumulation chains
for v in 1 2; do
  n=pl2f$( [ $v = 2 ] && echo 2 || true )
  /opt/rocm/bin/hipcc $F -DD2D_POLICY_L2_F32=$v -c csrc/policy_kernels.hip -o build/abl/policy_kernels_$n.o &
done
wait
for n in pl2f pl2f2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$n.so build/env_kernels.o \
    build/gae_kernels.o build/abl/policy_kernels_$n.o build/update_kernels.o build/gru_kernels.o build/abi.o
done
# r04 scheduling A/B: prng1 = Philox drawn before the tile MFMAs (D2D_POLICY_RNG_EARLY=1)
for spec in "prng1=-DD2D_POLICY_RNG_EARLY=1"; do
  n=${spec%%=*}
  /opt/rocm/bin/hipcc $F ${spec#*=} -c csrc/policy_kernels.hip -o build/abl/policy_kernels_$n.o &
done
wait
for n in prng1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$n.so build/env_kernels.o \
    build/gae_kernels.o build/abl/policy_kernels_$n.o build/update_kernels.o build/gru_kernels.o build/abi.o
done
