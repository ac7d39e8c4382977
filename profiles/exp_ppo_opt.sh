#!/bin/bash
# PPO optimizer (FlatAdamWGroups): GPU tests, then config 5 with it and with torch's AdamW.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 300 python -u -m pytest tests/test_ppo_gpu.py tests/test_agents.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for t in 0 1 0 1; do
  MZ_PPO_TORCH_ADAMW=$t timeout -k 10 240 python -u -m mazerl.train_ppo --envs 4096 --steps 600 | tail -1 | sed "s/^{/{\"torch_adamw\": $t, /" >> $out/ab.jsonl || exit 1
done
