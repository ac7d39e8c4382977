#!/bin/bash
# rocprofv3 kernel trace of the training leg alone (bench.py's win-rate half, 300 vector steps),
# for the per-stream breakdown in profiles/train_streams.py. Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 2 --train-steps 300 --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= > $O/kt.log 2>&1
