#!/bin/bash
# k_reset_done's reset chain: winner flags loaded once per group, the bank maze's meta words passed
# in registers, 32 loads in flight per lane in the bank copy (default) vs the previous kernel
# (profiles/_bin/rd_head.so): env / bank / checkpoint GPU tests, DDQN training A/B interleaved,
# a training trace (k_reset_done per vector step), then the k_step PMC passes (profiles/collect.sh).
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rdchain
mkdir -p $O
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for v in default rd_head default rd_head; do
  lib=$D; [ $v = default ] || lib=$PWD/profiles/_bin/$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 2 --train-steps 1200 --no-cpu-baseline --eval-mazes 64 --legs bits > $O/kt.log 2>&1
for f in $(find $O/kt -name '*kernel_trace.csv'); do python3 profiles/train_streams.py $f > $O/train_streams.json; rm -f $f; done
bash profiles/collect.sh
