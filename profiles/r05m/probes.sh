#!/bin/bash
# round 5: k_mcclendon phase probes at the current sources (MZ_MC_PROBE = k: return after phase k)
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in default 1 2 3 4 5 6 7; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_probes.jsonl || exit 1
done
