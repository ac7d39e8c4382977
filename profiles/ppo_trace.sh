#!/bin/bash
# rocprofv3 kernel stats of the config-5 PPO trainer (4,096 toroidal 17..79, 200 vector steps).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ppo_trace; mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 -m mazerl.train_ppo --envs 4096 --steps 200 --eval-mazes 64 > $O/kt.log 2>&1
