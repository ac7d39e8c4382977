#!/bin/bash
# round 5: McClendon phase B by jump pointers (parity tests + timing), k_mcclendon PMC passes
# (the whole kernel and the MZ_MC_PROBE=6 variant that stops before the hallway phase G), then the
# whole bench with best-of-6 training mazes, the global curriculum, cfg2 / cfg5 growth legs
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_schedule.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_timing.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
for lib in default p6; do
  if [ $lib = p6 ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp6.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d /tmp/mc_$lib/a -o run -- python3 profiles/exp_mc_prof.py r-prim > $O/pmc_${lib}_a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE -f csv -d /tmp/mc_$lib/b -o run -- python3 profiles/exp_mc_prof.py r-prim > $O/pmc_${lib}_b.log 2>&1 || exit 1
  for p in a b; do cp /tmp/mc_$lib/$p/*/run_counter_collection.csv $O/pmc_${lib}_$p.csv 2>/dev/null || find /tmp/mc_$lib/$p -name "*counter_collection.csv" -exec cp {} $O/pmc_${lib}_$p.csv \; ; done
done
unset MZ_LIB_OVERRIDE
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
