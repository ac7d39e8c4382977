#!/bin/bash
# (1) Where a cell-space Philox build's time goes: gen_rate at 65,536 x 81x81 with MZ_GPROBE
#     variants (profiles/_bin/gprobe_<v>.so: 1 no tables, 2 no distance field, 4 no goal scan).
# (2) Bank refill concurrency in training: MZ_BANK_WGS caps (profiles/_bin/gen_bank<w>.so) vs the
#     default (as many builds as fit), bench.py's DDQN training leg, interleaved.
# Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/genprobe
mkdir -p $O
B=$PWD/profiles/_bin
D=$PWD/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
for v in default 1 2 4 7; do
  lib=$D; [ $v = default ] || lib=$B/gprobe_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 120 python3 -u profiles/gen_rate.py --philox-81 | sed "s/^{/{\"gprobe\": \"$v\", /" >> $O/gen_rate.jsonl
done
for v in default bank1024 bank512 bank2048 default bank1024 bank512; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 --legs bits > $O/bench_$v.json
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); w=d['win_rate']; print(json.dumps({'lib': '$v', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy']}))" >> $O/train.jsonl
done
# (3) the same caps in config 5 (PPO, 4,096 toroidal 17..79: square-grid builds, 35 KB each)
export PYTHONPATH="$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
for v in default bank512 bank1024 default bank512 bank1024; do
  lib=$D; [ $v = default ] || lib=$B/gen_$v.so
  MZ_LIB_OVERRIDE=$lib timeout -k 10 300 python3 -u -m mazerl.train_ppo --envs 4096 --steps 600 > $O/cfg5_$v.jsonl 2> $O/cfg5_$v.err
  tail -1 $O/cfg5_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'train_env_steps_per_s': d['train_env_steps_per_s'], 'win_rate_greedy': d['win_rate_greedy']}))" >> $O/cfg5.jsonl
done
