#!/bin/bash
# Round profile collection on the GPU box (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats of a short headline bench (no training / CPU legs)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE of the same command
# Outputs under gpurun_out/prof/; profiles/summarize.py turns them into profiles/<tag>_*.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
ARGS="--steps 300 --warmup 30 --train-steps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py $ARGS > $O/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 bench.py $ARGS > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 bench.py $ARGS > $O/write.log 2>&1
