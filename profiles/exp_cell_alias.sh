#!/bin/bash
# Cell-space build with the distance array aliased on the carve list (8.5 KB of LDS at 81 x 81,
# default) vs separate (11.7 KB, profiles/_bin/gen_noalias.so = -DMZ_CELL_ALIAS=0): GPU tests,
# generation rates and the DDQN training leg, interleaved. Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/alias
mkdir -p $O
B=$PWD/profiles/_bin
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py \
  tests/test_gpu_dropin.py tests/test_metrics.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for v in default noalias default noalias; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 120 python3 -u profiles/gen_rate.py --philox-81 | sed "s/^{/{\"lib\": \"$v\", /" >> $O/gen_rate.jsonl
done
for v in default noalias default noalias; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
