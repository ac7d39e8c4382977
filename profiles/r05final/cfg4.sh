#!/bin/bash
# round 5: config 4 over 600 and 3,000 vector steps with the training wins per algorithm
set -o pipefail
O=gpurun_out/r05final
mkdir -p $O
export PYTHONUNBUFFERED=1
for n in 600 3000; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --train-steps 0 --curriculum-steps 0 \
    --no-cpu-baseline --config-legs cfg4 --cfg4-steps $n > $O/cfg4_$n.json 2> $O/cfg4_$n.err || exit 1
done
