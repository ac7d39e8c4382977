#!/bin/bash
# round 6: where the best-of-6 fill's time goes (kernel trace of exp_bestof_fill.py) and the lite
# carve kernel's SQ counters (occupancy, LDS waits, instruction mix)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06p
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_bestof_fill.py 2048 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY -f csv -d $O/pa -o run -- python3 profiles/exp_bestof_fill.py 2048 > $O/pa.log 2>&1 || { tail -20 $O/pa.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -f csv -d $O/pb -o run -- python3 profiles/exp_bestof_fill.py 2048 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
ls -R $O | head -30
