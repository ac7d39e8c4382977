#!/bin/bash
# round 6: config 5's growth leg trained longer — how far the instances grow
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06n
mkdir -p $O
export PYTHONUNBUFFERED=1
for n in 3000 8000; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --train-steps 0 \
    --curriculum-steps 0 --config-legs cfg5 --cfg5-modes growth --cfg5-steps $n --cfg-eval-mazes 300 \
    > $O/g$n.json 2> $O/g$n.err || { tail -20 $O/g$n.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/g$n.json').read().strip().splitlines()[-1]);g=d['configs']['cfg5_growth']
print(json.dumps({k:g.get(k) for k in ('vector_steps','seconds','env_steps_per_s','train_wins','instances_per_size_at_end','retired','stopped_at','win_rate_greedy','win_rate_greedy_best_of_6','seen_mazes_reference_protocol')}))"
done
