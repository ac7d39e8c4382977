#!/bin/bash
# round 5: k_mcclendon node arrays sized by the node count rounded to 64 (LDS 143 -> 120 KB at
# 81x81): McClendon tests, timing + checksum vs HEAD's kernel, then best-of-6 DDQN training vs
# HEAD's kernel (interleaved) — does LDS left free for the trainer's kernels on the refill's CUs
# show up in training throughput?
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || exit 1
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
