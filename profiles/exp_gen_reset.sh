#!/bin/bash
# Maze build from the carved tree (MZ_TREE_DIST: no level-synchronous BFS for Philox euclidean
# mazes) and k_reset_done's split groups (MZ_RD_SPLIT waves per 64 instances) + batched bank copy:
# GPU tests, generation rates and the DDQN training leg, A/B against variants built by
#   profiles/build_variant.sh profiles/_bin/gen_<variant>.so -D...   (VARIANTS="sq ..." below)
# (round 3: gen_bfs = -DMZ_TREE_DIST=0 -DMZ_RD_SPLIT=1, gen_tree_rd1 = -DMZ_RD_SPLIT=1;
#  then gen_sq = -DMZ_CELL_BUILD=0: the square-grid build instead of the cell-space one)
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-genreset}
mkdir -p $O
B=$PWD/profiles/_bin
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py \
  tests/test_mcclendon_gpu.py tests/test_metrics.py tests/test_gpu_dropin.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for v in default ${GEN_VARIANTS:-bfs}; do
  lib=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
  [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 120 python3 -u profiles/gen_rate.py | sed "s/^{/{\"lib\": \"$v\", /" >> $O/gen_rate.jsonl
done
for v in ${TRAIN_VARIANTS:-default tree_rd1 bfs default bfs}; do
  lib=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
  [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy'], 'gen': d['generation']['steady_mazes_per_s']}))" >> $O/train.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 2 --train-steps ${TRACE_STEPS:-300} --no-cpu-baseline --eval-mazes 64 > $O/kt.log 2>&1
for f in $(find $O/kt -name '*kernel_trace.csv'); do python3 profiles/train_streams.py $f > $O/train_streams.json; done
