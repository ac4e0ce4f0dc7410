# r03 precision A/B of the actor update kernel (lib/libd2dhip_<v>.so; timing with
# tools/gpu/ablate_update.py <v> ...): p3: the kernels before the three-way logits split (3940e31);
# s2: the current kernels with the two-way split in the logits; pk: split residuals on v_pk_add_f32
# instead of v_dot2c_f32_bf16; s2pk: both.
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../include -Icsrc"
OTHER="build/env_kernels.o build/gae_kernels.o build/policy_kernels.o build/gru_kernels.o build/abi.o"
git show 3940e31:d2d-ppo_amd/csrc/update_kernels.hip > build/abl/update_kernels_p3.hip
build() {  # name, source, extra flags
  /opt/rocm/bin/hipcc $F $3 -c $2 -o build/abl/upd_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$1.so $OTHER build/abl/upd_$1.o
}
build p3 build/abl/update_kernels_p3.hip "" &
build s2 csrc/update_kernels.hip "-DD2D_LOGITS_SPLIT3=0" &
build pk csrc/update_kernels.hip "-DD2D_SPLIT_DOT2=0" &
build s2pk csrc/update_kernels.hip "-DD2D_LOGITS_SPLIT3=0 -DD2D_SPLIT_DOT2=0" &
wait
