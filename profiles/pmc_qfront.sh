#!/bin/bash
# k_qfront (acting conv stem) counters: kernel trace + stats, then one rocprofv3 --pmc pass per
# counter group over profiles/exp_qfront.py. Usage (GPU box, repo root): profiles/pmc_qfront.sh <outdir>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1
mkdir -p "$out"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$out/kt" -o run -- python3 profiles/exp_qfront.py > "$out/kt.log" 2>&1
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp -f csv -d "$out/p$i" -o run -- python3 profiles/exp_qfront.py > "$out/p$i.log" 2>&1
  i=$((i+1))
done
