#!/bin/bash
# round 5: prim&kill walk with the mark's 5 x 5 window in registers — the generation tests, then
# Philox builds (meta hashes + rate) against HEAD's carve, interleaved
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_env.py tests/test_best_of_bank.py tests/test_bank.py > $O/tests.log 2>&1 || exit 1
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_gen_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 200 python -u profiles/gen_rate.py >> $O/gen_ab.jsonl || exit 1
done
