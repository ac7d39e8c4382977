#!/bin/bash
# round 5: McClendon without scratch (WSet as value selects): parity + timing + PMC; config 5's
# fixed-size leg with 1 vs 6 candidates (same seeds)
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_best_of_bank.py tests/test_difficulty.py tests/test_metrics.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_timing.jsonl || exit 1
MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp6.so timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_timing.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d /tmp/mc/a -o run -- python3 profiles/exp_mc_prof.py r-prim > $O/pmc_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE -f csv -d /tmp/mc/b -o run -- python3 profiles/exp_mc_prof.py r-prim > $O/pmc_b.log 2>&1 || exit 1
for p in a b; do find /tmp/mc/$p -name "*counter_collection.csv" -exec cp {} $O/pmc_$p.csv \; ; done
for c in 1 6; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --curriculum-steps 0 \
    --legs bits --config-legs cfg5 --cfg5-modes fixed --candidates $c > $O/cfg5_c$c.json 2> $O/cfg5_c$c.err || exit 1
done
