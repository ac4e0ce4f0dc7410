# r03 scheduling / indexing variants of the update kernels (lib/libd2dhip_<v>.so; timing A/B with
# tools/gpu/ablate_update.py <v> ...).  h: the r02 kernels (git HEAD~ copy in build/abl); i: division-free
# tile cursor; x / y: i + the max-ilp / iterative-ilp machine scheduler; z: i + 3 waves/SIMD budget.
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc"
OTHER="build/env_kernels.o build/gae_kernels.o build/policy_kernels.o build/gru_kernels.o build/abi.o"
build() {  # name, source, extra flags
  /opt/rocm/bin/hipcc $F $3 -c $2 -o build/abl/upd_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$1.so $OTHER build/abl/upd_$1.o
}
build h build/abl/update_kernels_head.hip "" &
build i csrc/update_kernels.hip "" &
build x csrc/update_kernels.hip "-mllvm -amdgpu-sched-strategy=max-ilp" &
build y csrc/update_kernels.hip "-mllvm -amdgpu-sched-strategy=iterative-ilp" &
build z csrc/update_kernels.hip "-DD2D_UPD_WAVES=3" &
wait
