#!/bin/bash
# An experiment library: the current objects of libmazerl.so with ONE source replaced by another
# version of it (a file path or a git revision's copy), into profiles/_bin/<name>.so (gitignored).
#   profiles/build_variant.sh <name> <csrc file name> <alt source path | git rev> [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; file=$2; alt=$3; shift 3
C=maze-solving-agent-gymnasium_amd/csrc
L=maze-solving-agent-gymnasium_amd/mazerl/_lib
src=$alt
if [ ! -f "$alt" ]; then src=/tmp/variant_$name.hip; git show "$alt:$C/$file" > $src; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I $C "$@" -c -o /tmp/variant_$name.o $src
mkdir -p profiles/_bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o profiles/_bin/$name.so $(ls $L/obj/*.o | grep -v "/$file.o") /tmp/variant_$name.o
echo profiles/_bin/$name.so
