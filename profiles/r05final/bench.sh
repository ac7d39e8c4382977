#!/bin/bash
# round 5 final: the driver's bench command (defaults: N = 1, its default steps and legs) and a
# longer config-4 leg (3,000 vector steps) for the per-algorithm training wins
set -o pipefail
O=gpurun_out/r05final
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --train-steps 0 --curriculum-steps 0 \
  --no-cpu-baseline --config-legs cfg4 --cfg4-steps 3000 > $O/cfg4_3000.json 2> $O/cfg4_3000.err || exit 1
