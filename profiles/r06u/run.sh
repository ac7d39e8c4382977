#!/bin/bash
# round 6: stream priorities with the capped refill — learner side stream and / or the acting
# stream at high priority (-1), the refill stream at the default; best-of-6 DDQN training
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06u
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in none learner act both none learner act both; do
  unset MZ_LEARNER_PRIORITY MZ_ACT_PRIORITY
  case $v in learner) export MZ_LEARNER_PRIORITY=-1;; act) export MZ_ACT_PRIORITY=-1;;
    both) export MZ_LEARNER_PRIORITY=-1 MZ_ACT_PRIORITY=-1;; esac
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" > $O/bench_$v.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'prio':'$v','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
