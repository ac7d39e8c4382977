#!/bin/bash
# Round profile collection on the GPU box (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats of a short headline bench per env-step leg (no training
#      / CPU legs; both legs launch the same k_step instantiation, so one leg per run)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE per leg (window: f32 Enrich window,
#      bits: the trainers' window-bits mode), one leg per pass so the k_step launches are that
#      leg's only
# Outputs under gpurun_out/prof/; profiles/summarize.py turns them into profiles/<tag>_* and the
# records of profiles/pmc_k_step.json.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
O=gpurun_out/prof
mkdir -p $O
ARGS="--steps 300 --warmup 30 --train-steps 0 --curriculum-steps 0 --config-legs= --no-cpu-baseline"
# the kernel trace with the bench's captured-graph replays; the counter passes with eager launches
# (the same k_step launch, one dispatch at a time under counter collection)
for leg in window bits; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$leg -o run -- python3 bench.py $ARGS --legs $leg > $O/kt_$leg.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch_$leg -o run -- python3 bench.py $ARGS --graph 0 --legs $leg > $O/fetch_$leg.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write_$leg -o run -- python3 bench.py $ARGS --graph 0 --legs $leg > $O/write_$leg.log 2>&1
done
