#!/bin/bash
# round 6: the DDQN learner update's kernels alone (batch 1,024)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06r
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 profiles/exp_update_kernels.py > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_update_kernels.py > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cat $O/plain.json
