#!/bin/bash
# round 6: the full default bench at the current sources (Philox ring, tuned learner GEMMs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
