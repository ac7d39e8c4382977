#!/bin/bash
# round 5, first GPU check: best-of-C generation / bank, the win schedule (new tests first), the
# whole GPU suite, then the cost of best-of-6 training mazes in the bench's DDQN win-rate leg
# (candidates 6 vs 1)
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_best_of_bank.py tests/test_schedule.py > $O/tests_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests_all.log 2>&1 && \
for c in 6 1; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates $c > $O/bench_c$c.json 2> $O/bench_c$c.err || exit 1
done
