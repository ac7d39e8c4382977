#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_greedy_rows.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/bench81.json 2> $out/bench81.err &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --dim 41 > $out/bench41.json 2> $out/bench41.err
