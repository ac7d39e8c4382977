#!/bin/bash
# k_step in the trainers' window-bits mode: MZ_PROBE decomposition (see exp_probes.sh) and the
# batch-size dependence of the launch time. Build: PROBES="0 1 2 4 8 64 128 256" profiles/exp_probes.sh build
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bitsprobe
mkdir -p $O
for v in 0 1 2 4 8 64 128 256 0; do
  timeout -k 10 120 python3 profiles/exp_autoreset.py --bits --lib profiles/_bin/probe_$v.so --warmup 300 --iters 2000 \
    | sed "s/^{/{\"probe\": $v, /" >> $O/probes.jsonl
done
for B in 16384 32768 65536 131072 262144; do
  timeout -k 10 120 python3 profiles/exp_autoreset.py --bits --envs $B --warmup 300 --iters 2000 >> $O/sizes.jsonl
done
