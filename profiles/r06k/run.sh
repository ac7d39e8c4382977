#!/bin/bash
# round 6: the learner's gradient collectives captured inside the update graph (one RCCL rank):
# equality with the two-graph path and the eager update, then the cost per update vs none
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06k
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u profiles/exp_update_collective.py > $O/update_collective.json 2> $O/update_collective.err || { tail -30 $O/update_collective.err; exit 1; }
tail -1 $O/update_collective.json
