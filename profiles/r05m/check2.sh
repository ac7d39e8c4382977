#!/bin/bash
# round 5: McClendon phase G — lane-path hallways spread over MZ_MC_LANE_WAVES waves (default 12;
# 4, 8, 16) vs the previous mapping (the first threads), interleaved, with the tests
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_best_of_bank.py > $O/tests2.log 2>&1 || exit 1
for lib in prev new lw4 lw8 lw16 prev new; do
  case $lib in new) unset MZ_LIB_OVERRIDE;; prev) export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so;;
    *) export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_$lib.so;; esac
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_lw.jsonl || exit 1
done
