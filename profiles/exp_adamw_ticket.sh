#!/bin/bash
# A/B of k_adamw's grid (libraries from profiles/_bin/adamw_<workgroups>x<threads>.so, built with
# -DMZ_ADAMW_MAXWG / -DMZ_ADAMW_TPB): the optimizer step alone, then the bench's DDQN training
# leg. Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/adamw2
mkdir -p $O
V="512x256 256x512 256x1024 128x1024 128x512"
for W in $V; do
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/adamw_$W.so timeout -k 10 120 python3 -u profiles/exp_adamw_ticket.py >> $O/alone.jsonl
done
for W in $V 512x256; do
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/adamw_$W.so timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$W.json
  python3 -c "import json,sys; d=json.load(open('$O/bench_$W.json')); w=d['win_rate']; print(json.dumps({'grid': '$W', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
