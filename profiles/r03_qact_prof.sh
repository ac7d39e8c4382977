# k_qact1 / k_qact2 kernel times and SQ counters (exp_qact.py: 28,180 listed rows + 65,536 rows)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_qact.py main > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -f csv -d $O/p0 -o run -- python3 profiles/exp_qact.py main > $O/p0.log 2>&1 || { tail -20 $O/p0.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $O/p1 -o run -- python3 profiles/exp_qact.py main > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
grep -E "k_qact" $O/kt/run_kernel_stats.csv | cut -c1-160
