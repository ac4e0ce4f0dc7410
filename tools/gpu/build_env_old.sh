# A/B variant: the env kernels as of commit 4a3184b (before comb_step / the fused slot / the bf16 state rows),
# linked with the current objects -> lib/libd2dhip_envold.so (D2D_LIB_VARIANT=envold, D2D_ALLOW_ABLATION=1).
# d2d_comb_policy_fused_step is a stub there (D2D_EUNSUPPORTED): env / rollout legs only.
set -e
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
git show 4a3184b:d2d-ppo_amd/csrc/env_kernels.hip > build/abl/env_kernels_old.hip
cat > build/abl/fused_stub.cpp <<'EOC'
#include "d2d_hip.h"
extern "C" int d2d_comb_policy_fused_step(const d2d_env_desc*, const d2d_env_state*, const void*, const d2d_env_out*,
                                          int32_t, uint32_t, const d2d_mlp_desc*, uint32_t, int32_t, void*, float*,
                                          void*) { return D2D_EUNSUPPORTED; }
EOC
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include -Icsrc"
/opt/rocm/bin/hipcc $F -c build/abl/env_kernels_old.hip -o build/abl/env_kernels_old.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -I../include -c build/abl/fused_stub.cpp -o build/abl/fused_stub.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_envold.so build/abl/env_kernels_old.o \
  build/abl/fused_stub.o build/gae_kernels.o build/policy_kernels.o build/update_kernels.o build/gru_kernels.o \
  build/critic_kernels.o build/abi.o
