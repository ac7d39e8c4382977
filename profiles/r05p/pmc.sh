#!/bin/bash
# round 5: where a serial build chain / k_mcclendon spends its cycles — SQ instruction and wait
# counters for k_build (Philox r-prim / dfs / prim&kill, 65,536 x 81x81) and k_mcclendon (6,000
# 81x81 candidates per algorithm + toroidal), two counter passes each. Raw CSVs stay in /tmp; the
# per-dispatch summary goes to gpurun_out/r05p/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
n=0
for prog in "profiles/gen_rate.py --philox-81" "profiles/exp_mcclendon_wg.py"; do
  n=$((n + 1))
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    timeout -s KILL 300 rocprofv3 --pmc $C -f csv -d /tmp/pmc_${n}_$p -o run -- python3 $prog > $O/run_${n}_$p.log 2>&1 || exit 1
    python3 profiles/r05p/pmc_sum.py /tmp/pmc_${n}_$p >> $O/pmc.jsonl || exit 1
  done
done
