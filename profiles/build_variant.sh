#!/bin/bash
# Build libmazerl.so with extra compile flags into profiles/_bin/<name>.so (A/B variants).
# usage: profiles/build_variant.sh <name> <flags...>
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/maze-solving-agent-gymnasium_amd/csrc
O=/tmp/variant_$name
mkdir -p $O $ROOT/profiles/_bin
objs=()
for f in mz_env.hip mz_api.hip mz_difficulty.hip mz_qnet.hip mz_metrics.hip mz_stem.hip mz_optim.hip \
         mz_trainer.hip mz_ppo.hip mz_qact.hip mz_mcclendon.hip mz_screen.hip; do
  extra=""
  [ $f = mz_qnet.hip ] && extra="-ffinite-math-only"
  [ $f = mz_qact.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $extra "$@" -c -o $O/$f.o $C/$f &
  objs+=($O/$f.o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/profiles/_bin/$name.so "${objs[@]}"
echo $ROOT/profiles/_bin/$name.so
