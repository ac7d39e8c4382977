#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only beside --pmc) of the
# k_step decomposition runs in profiles/exp_kstep.py. Usage: profiles/pmc_kstep.sh <outdir> [exp args]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; shift
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$out/p$i" -o run -f csv -- python3 profiles/exp_kstep.py --iters 30 "$@" > "$out/p$i.log" 2>&1
  i=$((i+1))
done
