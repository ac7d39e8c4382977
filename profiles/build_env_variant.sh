#!/bin/bash
# A/B build of libmazerl.so with extra compile flags for mz_env.hip (timing probes):
#   profiles/build_env_variant.sh <out.so> -DFLAG ...   (run after mazerl._build has built obj/)
set -e
out=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/maze-solving-agent-gymnasium_amd/mazerl/_lib/obj
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall "$@" \
  -I$R/maze-solving-agent-gymnasium_amd/csrc -c -o $tmp/env.o $R/maze-solving-agent-gymnasium_amd/csrc/mz_env.hip
objs=$(ls $O/*.o | grep -v mz_env.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $tmp/env.o $objs
rm -rf $tmp
