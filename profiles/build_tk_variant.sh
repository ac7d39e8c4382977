#!/bin/bash
# A/B build of libmazerl.so with the learner's last-workgroup tickets at G groups (mz_learner.h
# MZ_TK_G; 1 = one same-address ticket): profiles/build_tk_variant.sh <out.so> <G>
set -e
out=$1; G=$2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/maze-solving-agent-gymnasium_amd/mazerl/_lib/obj
tmp=$(mktemp -d)
for src in mz_optim.hip mz_trainer.hip mz_api.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -DMZ_TK_G=$G \
    -c -o $tmp/$src.o $R/maze-solving-agent-gymnasium_amd/csrc/$src &
done
wait
objs=$(ls $O/*.o | grep -v -e "/mz_optim.hip.o" -e "/mz_trainer.hip.o" -e "/mz_api.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $tmp/*.o $objs
rm -rf $tmp
