#!/bin/bash
# AdamW step count advanced by a one-thread launch before k_adamw (no per-workgroup ticket, 2,048
# workgroups of 256; default) vs the ticketed k_adamw (profiles/_bin/aw_ticket.so,
# -DMZ_ADAMW_PREINC=0), and k_qact1 with 8-wave workgroups (qw8.so, -DMZ_QACT_WAVES=8) and
# k_reset_done with one wave per group (rd1.so, -DMZ_RD_SPLIT=1): optimizer / learner /
# checkpoint GPU tests, then DDQN training A/B interleaved.
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/adamw
mkdir -p $O
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 600 python3 -u -m pytest tests/test_flat_optim.py tests/test_learner.py tests/test_learner_graph.py \
  tests/test_learner_overlap.py tests/test_trainer_kernels.py tests/test_checkpoint_gpu.py tests/test_gpu_distributed.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for v in default aw_ticket qw8 rd1 default aw_ticket qw8 rd1; do
  lib=$D; [ $v = default ] || lib=$PWD/profiles/_bin/$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
