#!/bin/bash
# round 5: (1) McClendon hallway-0 terms in parallel: tests + timing vs HEAD's kernel; (2) best-of-6
# training with the acting (and learner) streams at high priority and the bank refills at the
# default one — the refills' McClendon workgroups hold a CU's LDS for milliseconds
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || exit 1
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
unset MZ_LIB_OVERRIDE
for v in base act both base act both; do
  case $v in base) unset MZ_ACT_PRIORITY MZ_LEARNER_PRIORITY;;
    act) export MZ_ACT_PRIORITY=-1; unset MZ_LEARNER_PRIORITY;;
    both) export MZ_ACT_PRIORITY=-1 MZ_LEARNER_PRIORITY=-1;; esac
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$v.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'variant':'$v','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/prio.jsonl
done
