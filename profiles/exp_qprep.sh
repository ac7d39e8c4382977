#!/bin/bash
# QAct: tiled coalesced weight preparation (k_qact_prep1/2) + k_qact2 over 128 rows per workgroup
# (default) vs the same with 64 rows (profiles/_bin/qact2_64.so, -DMZ_QACT2_ROWS=64) vs the
# previous mz_qact.hip (profiles/_bin/qprep_old.so: per-element gather, 64 rows): every GPU test,
# the DDQN training leg and bench's q_head timings interleaved, then the k_step PMC passes of
# profiles/collect.sh for the current sources.
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qprep
mkdir -p $O
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for v in default qact2_64 qprep_old default qact2_64 qprep_old; do
  lib=$D; [ $v = default ] || lib=$PWD/profiles/_bin/$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; q=d['q_head']['x3']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy'], 'qhead_all_ms': q['all_rows']['ms'], 'qhead_greedy_ms': q['greedy_rows']['ms'], 'greedy_rows': q['greedy_rows']['rows']}))" >> $O/train.jsonl
done
bash profiles/collect.sh
