#!/bin/bash
# Multi-size maze bank: bank / PPO / trainer tests, then config 5 with and without the bank.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 400 python -u -m pytest tests/test_bank.py tests/test_ppo_gpu.py tests/test_trainer_kernels.py tests/test_greedy_rows.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for f in "" "--no-bank" "" "--no-bank"; do
  timeout -k 10 240 python -u -m mazerl.train_ppo --envs 4096 --steps 600 $f | tail -1 | sed "s/^{/{\"flags\": \"$f\", /" >> $out/ab.jsonl || exit 1
done
