#!/bin/bash
# Trainer bookkeeping kernels: GPU tests, then an A/B of bench.py's training leg (fused
# bookkeeping + ring push vs torch ops; both with the greedy-row acting). Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_trainer_kernels.py tests/test_greedy_rows.py tests/test_learner_overlap.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for f in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fused-bookkeeping $f >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
