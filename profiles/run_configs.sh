#!/bin/bash
# The other BASELINE.json configs' training runs on one GPU (per-GPU shares of the 8-GPU ones), and
# a 2-rank rehearsal of bench.py's N>1 path (gloo, both ranks on this GPU). Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
# cfg2: 4,096 x 15x15 r-prim DQN; cfg4 per-GPU share: 8,192 x 81x81 mixed DDQN (4 updates of 512 per vector step)
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 400 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/configs.jsonl &&
timeout -k 10 240 python -u -m mazerl.train --envs 8192 --dim 81 --algo mixed --variant ddqn --steps 600 --batch 512 --updates-per-step 4 --log-every 0 | tail -1 >> $out/configs.jsonl &&
timeout -k 10 240 python -u -m mazerl.train_ppo --envs 4096 --steps 600 | tail -1 >> $out/configs.jsonl &&
MZ_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --envs 16384 --steps 100 --warmup 10 --train-steps 60 --eval-mazes 100 > $out/rehearsal_2rank.txt 2>&1
