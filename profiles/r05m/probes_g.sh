#!/bin/bash
# round 5: k_mcclendon phase-G sub-probes (71 / 72: return after G's member lists / G1's
# classification; 73 / 74: the whole kernel without the lane path / the wave queue)
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in default 71 72 73 74 7; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_probes_g.jsonl || exit 1
done
