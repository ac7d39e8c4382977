#!/bin/bash
# A/B build of libmazerl.so with extra compile flags for one source (timing experiments):
#   profiles/build_src_variant.sh <out.so> <source.hip> -DFLAG ...   (after mazerl._build has built obj/)
set -e
out=$1; src=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/maze-solving-agent-gymnasium_amd/mazerl/_lib/obj
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall "$@" \
  -c -o $tmp/v.o $R/maze-solving-agent-gymnasium_amd/csrc/$src
objs=$(ls $O/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $tmp/v.o $objs
rm -rf $tmp
