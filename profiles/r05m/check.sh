#!/bin/bash
# round 5: McClendon lane path with a node-key table and batched neighbour loads — the McClendon
# tests, then outputs + timing against the previous lane path (lib_mc_prev), interleaved, and the
# phase probes (6: before phase G, 7: after it)
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || exit 1
for lib in prev new prev new mcp6 mcp7; do
  case $lib in new) unset MZ_LIB_OVERRIDE;; prev) export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so;;
    *) export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so;; esac
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
