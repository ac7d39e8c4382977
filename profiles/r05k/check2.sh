#!/bin/bash
# round 5: which kernels the K-update graph replays that the single-update replays do not
# (rocprofv3 kernel stats of the same 200-step live run, MZ_K_BLOCK=0 vs 1)
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for kb in 0 1; do
  MZ_K_BLOCK=$kb timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/kb$kb -o run -- python3 profiles/r05f/kblock_repro.py new 200 > $O/kb_trace$kb.log 2>&1 || exit 1
  cp /tmp/kb$kb/run_kernel_stats.csv $O/kb${kb}_kernel_stats.csv
done
