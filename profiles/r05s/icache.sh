#!/bin/bash
# round 5: is k_mcclendon (84 KB of code) instruction-fetch bound? the counters the box offers for
# the instruction cache, then one pass of them over the McClendon timing experiment (k_mcclendon
# dispatches summed per algorithm by profiles/r05p/pmc_sum.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > /tmp/avail.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*\|SQ_INST_CYCLES[A-Z_0-9]*\|SQ_WAIT_[A-Z_0-9]*" /tmp/avail.txt | sort -u > $O/icache_counters.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -f csv -d /tmp/pmc_ic -o run -- python3 profiles/exp_mcclendon_wg.py > $O/icache_run.log 2>&1 || exit 1
python3 profiles/r05p/pmc_sum.py /tmp/pmc_ic > $O/icache_pmc.jsonl
