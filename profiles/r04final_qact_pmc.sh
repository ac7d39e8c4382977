# round 4 (final sources): k_qconv / k_qfc1 / k_qact2 PMC passes at 65,536 rows with dropout (profiles/exp_qact.py prof):
# kernel trace + stall / instruction-mix counters + HBM bytes, one rocprofv3 pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q=gpurun_out/r04final_qpmc; mkdir -p $Q
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $Q/kt -o run -- python3 profiles/exp_qact.py prof > $Q/kt.log 2>&1 || { tail -20 $Q/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $Q/a -o run -- python3 profiles/exp_qact.py prof > $Q/a.log 2>&1 || { tail -20 $Q/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE -f csv -d $Q/b -o run -- python3 profiles/exp_qact.py prof > $Q/b.log 2>&1 || { tail -20 $Q/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $Q/fetch -o run -- python3 profiles/exp_qact.py prof > $Q/fetch.log 2>&1 || { tail -20 $Q/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $Q/write -o run -- python3 profiles/exp_qact.py prof > $Q/write.log 2>&1 || { tail -20 $Q/write.log; exit 1; }
echo pmc-ok
