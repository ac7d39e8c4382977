#!/bin/bash
# A/B of k_colsum's workgroup width (libraries from profiles/_bin/colsum_<quads>.so, built with
# -DMZ_COLSUM_CQ: 4 x quads columns and 64 x quads threads per workgroup, the same summation
# order): the colsum test, then the bench's DDQN training leg. Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/colsum
mkdir -p $O
for W in 4 1; do
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/colsum_$W.so timeout -k 10 120 python3 -u -m pytest tests/test_graph_linear.py -m gpu -x -q --timeout 60 --timeout-method thread >> $O/tests.log 2>&1
done
for W in 16 4 1 16 4 1; do
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/colsum_$W.so timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$W.json
  python3 -c "import json,sys; d=json.load(open('$O/bench_$W.json')); w=d['win_rate']; print(json.dumps({'quads': $W, 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
