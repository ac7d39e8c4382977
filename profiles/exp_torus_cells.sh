#!/bin/bash
# Toroidal Philox builds in cell space + bit-parallel torus BFS (default) vs the square-grid build
# (profiles/_bin/gen_sq.so = -DMZ_CELL_BUILD=0): GPU tests, generation rates, config 5 (PPO).
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/torus
mkdir -p $O
B=$PWD/profiles/_bin
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py \
  tests/test_mcclendon_gpu.py tests/test_metrics.py tests/test_gpu_dropin.py tests/test_ppo_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for v in default sq; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 120 python3 -u profiles/gen_rate.py | sed "s/^{/{\"lib\": \"$v\", /" | grep philox >> $O/gen_rate.jsonl
done
export PYTHONPATH="$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
for v in default sq default sq; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u -m mazerl.train_ppo --envs 4096 --steps 600 > $O/cfg5_$v.jsonl 2> $O/cfg5_$v.err
  tail -1 $O/cfg5_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'train_env_steps_per_s': d['train_env_steps_per_s'], 'win_rate_greedy': d['win_rate_greedy']}))" >> $O/cfg5.jsonl
done
