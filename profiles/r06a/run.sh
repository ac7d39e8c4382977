#!/bin/bash
# round 6, first GPU pass: the screen / pipeline tests, then best-of-6 fill timing A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_screen_gpu.py tests/test_best_of_bank.py > gpurun_out/r06a/tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06a/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 > gpurun_out/r06a/fill_new.jsonl 2>&1 || exit 1
MZ_LIB_OVERRIDE=profiles/_bin/lib_r05.so timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 > gpurun_out/r06a/fill_old.jsonl 2>&1 || exit 1
cat gpurun_out/r06a/fill_new.jsonl gpurun_out/r06a/fill_old.jsonl
