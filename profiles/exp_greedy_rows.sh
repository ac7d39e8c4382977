#!/bin/bash
# A/B of the acting forward over the greedy rows only vs every instance, on bench.py's training
# leg (65,536 x 81x81 r-prim DDQN, 2,400 vector steps + evaluation). Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_greedy_rows.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for g in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --greedy-rows $g >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
