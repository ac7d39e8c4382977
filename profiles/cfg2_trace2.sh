#!/bin/bash
# Round 4: config 2 (4,096 x 15x15 r-prim DQN, one update of 2,048 per vector step) traced again
# after the k_reset_done change (waves per group sized for >= 1,024 waves), and re-measured.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/kt -o run -- python3 -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 300 --batch 2048 --updates-per-step 1 --log-every 0 --eval-mazes 64 > $out/kt.log 2>&1 &&
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 1600 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/cfg2.jsonl
