#!/bin/bash
# A/B: the training leg's acting / env stream at high priority (MZ_ACT_PRIORITY=-1) vs default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
for p in -1 none -1 none; do
  if [ $p = none ]; then unset MZ_ACT_PRIORITY; else export MZ_ACT_PRIORITY=$p; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"prio\": \"$p\", /" >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
