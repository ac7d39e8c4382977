#!/bin/bash
# DDQN at the reference's own constant-size script size (41x41 grid = 20x20 cells,
# training_examples/.../costant_sizes/test_ddqn.py:20) — for the README's published win-rates.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
for steps in 600 2400; do
  timeout -k 10 300 python -u -m mazerl.train --envs 65536 --dim 41 --variant ddqn --steps $steps --batch 1024 --log-every 0 | tail -1 >> $out/ref_size.jsonl || exit 1
done
timeout -k 10 300 python -u -m mazerl.train --envs 65536 --dim 41 --variant dqn --steps 2400 --batch 1024 --log-every 0 | tail -1 >> $out/ref_size.jsonl
