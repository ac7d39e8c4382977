#!/bin/bash
# round 6: screen first-child by pointer jumping, division-free carve neighbours: tests, fill rate, kernel mix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_screen_gpu.py \
  tests/test_best_of_bank.py tests/test_build_algorithms.py tests/test_bank.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
cat $O/fill.jsonl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fill -- python3 profiles/exp_bestof_fill.py 2048 > $O/prof.log 2>&1 || exit 1
