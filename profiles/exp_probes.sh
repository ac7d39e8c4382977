#!/bin/bash
# k_step time decomposition: each MZ_PROBE variant (mz_env.hip) removes one piece of the step
# (results wrong — timing only), timed by exp_autoreset.py in the bench loop's steady state.
#   build (CPU container):  profiles/exp_probes.sh build
#   run (GPU box):          profiles/exp_probes.sh run <outdir>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS="${PROBES:-0 1 2 4 8 16 32 64 128 256 257 34 335 367}"
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    "$R/profiles/build_variant.sh" "$R/profiles/_bin/probe_$v.so" -DMZ_PROBE=$v &
  done
  wait
  [ -n "$NO_UBENCH" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o "$R/profiles/_bin/ubench_store" "$R/profiles/ubench_store.hip"
  exit 0
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$2; mkdir -p "$out"
timeout -k 10 60 profiles/_bin/ubench_store 4096 200 > "$out/ubench_store.jsonl"
for v in $VARIANTS; do
  timeout -k 10 120 python3 profiles/exp_autoreset.py --lib profiles/_bin/probe_$v.so --warmup 300 --iters 1000 \
    | sed "s/^{/{\"probe\": $v, /" >> "$out/probes.jsonl"
done
