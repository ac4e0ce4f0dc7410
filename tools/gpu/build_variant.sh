# A/B variant of one translation unit with extra defines -> lib/libd2dhip_<name>.so (D2D_LIB_VARIANT=<name>,
# D2D_ALLOW_ABLATION=1), linked with the product objects of the others.
# usage: bash tools/gpu/build_variant.sh <name> <unit: env_kernels|policy_kernels|update_kernels|...> -DMACRO=VALUE ...
set -e
NAME="$1"; UNIT="$2"; shift 2
cd "$(dirname "$0")/../../d2d-ppo_amd"
mkdir -p build/abl lib
EXTRA=""; [ "$UNIT" = update_kernels ] && EXTRA="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off $EXTRA --offload-arch=gfx950 -I../include -Icsrc "$@" \
  -c csrc/$UNIT.hip -o build/abl/${UNIT}_$NAME.o
OBJS=""
for u in env_kernels gae_kernels policy_kernels update_kernels gru_kernels critic_kernels; do
  if [ "$u" = "$UNIT" ]; then OBJS="$OBJS build/abl/${UNIT}_$NAME.o"; else OBJS="$OBJS build/$u.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libd2dhip_$NAME.so $OBJS build/abi.o
