#!/bin/bash
# round 5: config 4 (8,192 mixed-algorithm 81x81 instances per GPU, DDQN
# 4 x 512) trained 10,000 and 30,000 vector steps — does the learner ever win dfs / prim&kill
# training episodes, and what greedy win-rate per algorithm follows
set -o pipefail
O=gpurun_out/r05c4
mkdir -p $O
export PYTHONUNBUFFERED=1
for n in 10000 30000; do
  timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --legs bits --train-steps 0 --curriculum-steps 0 \
    --no-cpu-baseline --config-legs cfg4 --cfg4-steps $n > $O/cfg4_$n.json 2> $O/cfg4_$n.err || { tail -5 $O/cfg4_$n.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/cfg4_$n.json').read().strip().splitlines()[-1]);c=d['configs']['cfg4']
print(json.dumps({'steps':$n,'env_steps_per_s':c['env_steps_per_s'],'train_wins_by_algorithm':c.get('train_wins_by_algorithm'),'greedy_by_algorithm':c['win_rate_reference_protocol']['greedy_by_algorithm'],'greedy':c['win_rate_reference_protocol']['greedy']}))"
done
