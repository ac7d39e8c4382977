#!/bin/bash
# Round 4 (VERDICT next 9): rocprofv3 kernel trace of config 2's training loop (4,096 x 15x15
# r-prim DQN, the run_configs.sh settings) for the per-stream breakdown (profiles/train_streams.py),
# then config 2 re-measured with one update of 2,048 per vector step (the same samples per vector
# step as 4 updates of 512). Run under gpurun from the repo root: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/kt -o run -- python3 -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 300 --batch 512 --updates-per-step 4 --log-every 0 --eval-mazes 64 > $out/kt.log 2>&1 &&
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 400 --batch 512 --updates-per-step 4 --log-every 0 | tail -1 >> $out/cfg2.jsonl &&
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 400 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/cfg2.jsonl &&
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 1600 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/cfg2.jsonl &&
timeout -k 10 240 python -u -m mazerl.train --envs 8192 --dim 81 --algo mixed --variant ddqn --steps 600 --batch 512 --updates-per-step 4 --log-every 0 | tail -1 >> $out/cfg4.jsonl &&
timeout -k 10 240 python -u -m mazerl.train --envs 8192 --dim 81 --algo mixed --variant ddqn --steps 600 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/cfg4.jsonl
