#!/bin/bash
# round 6: the DDQN update's kernels alone at config 4's batch (512) and config 2's (2,048)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06r2
mkdir -p $O
for b in 512 2048; do
  timeout -k 10 200 python3 profiles/exp_update_kernels.py $b > $O/plain_$b.json 2> $O/plain_$b.err || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$b -o run -- python3 profiles/exp_update_kernels.py $b > $O/kt_$b.log 2>&1 || { tail -20 $O/kt_$b.log; exit 1; }
done
cat $O/plain_*.json
