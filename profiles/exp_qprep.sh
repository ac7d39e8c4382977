#!/bin/bash
# QAct weight preparation: tiled coalesced k_qact_prep1/2 (default) vs the per-element gather
# (profiles/_bin/qprep_old.so, the previous mz_qact.hip): every GPU test, the DDQN training leg
# interleaved, then the k_step PMC passes of profiles/collect.sh for the current sources.
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qprep
mkdir -p $O
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for v in default old default old; do
  lib=$D; [ $v = default ] || lib=$PWD/profiles/_bin/qprep_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
bash profiles/collect.sh
