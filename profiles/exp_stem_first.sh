#!/bin/bash
# Acting stem issued before the greedy-row count sync (reads the count on the device): tests,
# then bench.py's training leg twice. Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_greedy_rows.py tests/test_trainer_kernels.py tests/test_qfront.py tests/test_learner_overlap.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for f in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
