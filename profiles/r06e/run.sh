#!/bin/bash
# round 6: the full default bench (new legs: cfg1, seen / infer protocols, 30,000-step cfg4,
# resized per-instance curriculum leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
