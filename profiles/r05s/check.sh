#!/bin/bash
# round 5: k_mcclendon's lane path from occupancy masks (MZ_MC_LANE2): McClendon tests, timing +
# checksum vs HEAD's kernel (interleaved)
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || exit 1
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
