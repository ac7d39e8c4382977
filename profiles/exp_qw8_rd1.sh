#!/bin/bash
# DDQN training A/B after the cell-space builds changed the CU contention: k_qact1 with 8-wave
# workgroups (profiles/_bin/qw8.so, -DMZ_QACT_WAVES=8; round 3 measured it slower in training with
# the 35 KB builds beside it) and k_reset_done with one wave per 64-instance group
# (profiles/_bin/rd1.so, -DMZ_RD_SPLIT=1) vs the default, interleaved. Run under gpurun.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qw8rd1
mkdir -p $O
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
for v in default qw8 rd1 default qw8 rd1 default qw8; do
  lib=$D; [ $v = default ] || lib=$PWD/profiles/_bin/$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; q=d['q_head']['x3']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy'], 'qhead_all_ms': q['all_rows']['ms']}))" >> $O/train.jsonl
done
