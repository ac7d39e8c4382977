#!/bin/bash
# Q-head MFMA evidence: rocprofv3 kernel trace + stats, then one --pmc pass for the MFMA counters
# (bf16 / f32 matrix ops issued, MFMA busy cycles, GPU-active cycles) of profiles/exp_qhead.py.
# Usage (GPU box, repo root): profiles/pmc_qhead.sh <outdir>; then profiles/summarize_qhead.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1
mkdir -p "$out"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$out/kt" -o run -- python3 profiles/exp_qhead.py > "$out/kt.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$out/mfma" -o run -- python3 profiles/exp_qhead.py > "$out/mfma.log" 2>&1
