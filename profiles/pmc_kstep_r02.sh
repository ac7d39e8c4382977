#!/bin/bash
# k_step instruction / wait counters in the bench loop's steady state (profiles/exp_autoreset.py),
# one rocprofv3 --pmc pass per group. Usage (GPU box, repo root): profiles/pmc_kstep_r02.sh <outdir>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1
mkdir -p "$out"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -f csv -d "$out/p$i" -o run -- python3 profiles/exp_autoreset.py --warmup 100 --iters 100 > "$out/p$i.log" 2>&1
  i=$((i+1))
done
