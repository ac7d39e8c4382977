#!/bin/bash
# round 5: K-update graph nondeterminism — the current package with MZ_K_BLOCK=0 twice and =1
# twice (2,400 vector steps, the round-4 curriculum leg), a source-net digest every 100 steps
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export PYTHONUNBUFFERED=1
for kb in 0 0 1 1; do
  MZ_K_BLOCK=$kb timeout -k 10 400 python -u profiles/r05f/kblock_repro.py new >> $O/kblock.jsonl 2>> $O/kblock.err || exit 1
done
