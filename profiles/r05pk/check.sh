#!/bin/bash
# round 5: Philox r-prim candidate builds 4 per wave (k_cand_build_rprim): generation / bank tests,
# the bank fill rate and the best-of-6 DDQN training leg vs the committed library (interleaved)
set -o pipefail
O=gpurun_out/r05pk
mkdir -p $O
export PYTHONUNBUFFERED=1
PREV=profiles/_bin/headwt/maze-solving-agent-gymnasium_amd/mazerl/_lib/libmazerl.so
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_best_of_bank.py \
  tests/test_bank.py tests/test_schedule.py tests/test_build_algorithms.py tests/test_determinism_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=$PREV; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 200 python -u profiles/exp_bank_fill_time.py >> $O/fill.jsonl || exit 1
done
cat $O/fill.jsonl
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=$PREV; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs cfg2 --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate'];c=d['configs']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6'],'cfg2':c['cfg2']['env_steps_per_s'],'cfg2_greedy':c['cfg2']['win_rate_greedy']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
