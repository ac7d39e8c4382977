#!/bin/bash
# rocprofv3 kernel stats of the acting Q-head forward alone (65,536 instances, exp_qhead.py act).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qhead_trace; mkdir -p $O
QH_ITERS=50 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_qhead.py act > $O/kt.log 2>&1
