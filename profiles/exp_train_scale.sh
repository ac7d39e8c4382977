#!/bin/bash
# Is the training loop host-bound? Training throughput at 32,768 / 65,536 / 131,072 instances:
# vector steps/s staying flat while the GPU work per step doubles means the Python issue rate sets it.
for B in 32768 65536 131072; do
  timeout -k 10 200 python3 bench.py --envs $B --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 200 2>/dev/null \
   | python3 -c "import json,sys; d=json.load(sys.stdin); w=d['win_rate']; print(json.dumps({'envs': $B, 'train_env_steps_per_s': w['train_env_steps_per_s'], 'vector_steps_per_s': w['train_env_steps_per_s'] / $B, 'seconds': w['train_seconds_steady']}))" || exit 1
done
