#!/bin/bash
# PPO heads' first layers as one GEMM (_TwinFirstLayer): PPO tests, then config 5 with and
# without it (MZ_PPO_TWIN=0), twice each. Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
timeout -k 10 400 python -u -m pytest tests/test_ppo_gpu.py tests/test_agents.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for t in 1 0 1 0; do
  MZ_PPO_TWIN=$t timeout -k 10 240 python -u -m mazerl.train_ppo --envs 4096 --steps 600 | tail -1 | sed "s/^{/{\"twin\": $t, /" >> $out/ab.jsonl || exit 1
done
