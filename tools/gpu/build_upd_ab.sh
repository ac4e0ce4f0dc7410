# r04 A/B builds of the MLP update kernels (lib/libd2dhip_<v>.so; timing with tools/gpu/ablate_update.py <v> ...):
#   sub2: split residuals as v_perm / v_and + a scalar v_sub_f32 (D2D_SPLIT_DOT2=2) instead of v_dot2c_f32_bf16
# usage: bash tools/gpu/build_upd_ab.sh [variant=flags ...]
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc"
OTHER="build/env_kernels.o build/gae_kernels.o build/policy_kernels.o build/gru_kernels.o build/abi.o"
build() {  # name, extra flags
  /opt/rocm/bin/hipcc $F $2 -c csrc/update_kernels.hip -o build/abl/upd_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$1.so $OTHER build/abl/upd_$1.o
}
if [ $# -eq 0 ]; then set -- "sub2=-DD2D_SPLIT_DOT2=2"; fi
for spec in "$@"; do
  build "${spec%%=*}" "${spec#*=}" &
done
wait
