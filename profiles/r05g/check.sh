#!/bin/bash
# round 5: (1) McClendon phase G with a lane path (one hallway per lane) beside the wave path:
# the difficulty / metrics / best-of tests, then outputs + timing against the previous library
# (profiles/_bin/lib_mc_old.so), interleaved; (2) k_qconv patch rows 20: Q-value checksum and
# timing against the round-4 library; (4) training throughput with
# best-of-6 training mazes; (5) the sharded optimizer step (reduce-scatter + shard AdamW +
# all-gather) and what the collectives add to an update over one-rank RCCL
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_difficulty.py tests/test_metrics.py tests/test_best_of_bank.py \
  > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py tests/test_learner.py tests/test_learner_graph.py tests/test_flat_optim.py \
  tests/test_checkpoint_gpu.py tests/test_head_loss.py > $O/tests_learner.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/exp_update_collective.py > $O/update_collective.json 2> $O/update_collective.err || exit 1
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
# r04 (patch rows 17, LUT), pr20 (rows 20, no LUT, MFMA results in AGPRs), new (+ VGPR form)
for lib in old pr20 new new pr20; do
  case $lib in old) export MZ_LIB_OVERRIDE=profiles/_bin/lib_qact_old.so;;
    pr20) export MZ_LIB_OVERRIDE=profiles/_bin/lib_qact_pr20.so;; *) unset MZ_LIB_OVERRIDE;; esac
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py > $O/qact_checksum_$lib.json || exit 1
  timeout -k 10 200 python -u profiles/exp_qact.py $lib >> $O/qact_timing.jsonl || exit 1
done
unset MZ_LIB_OVERRIDE
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
Q=/tmp/qpmc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $Q/kt -o run -- python3 profiles/exp_qact.py prof > $O/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $Q/a -o run -- python3 profiles/exp_qact.py prof > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE -f csv -d $Q/b -o run -- python3 profiles/exp_qact.py prof > $O/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $Q/fetch -o run -- python3 profiles/exp_qact.py prof > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $Q/write -o run -- python3 profiles/exp_qact.py prof > $O/write.log 2>&1 || exit 1
python3 profiles/summarize_qact_pmc.py $Q > $O/qact_pmc.json
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_adamw_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 120 python -u profiles/exp_adamw_ticket.py >> $O/adamw_ab.jsonl || exit 1
done
unset MZ_LIB_OVERRIDE
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --curriculum-steps 0 \
  --config-legs "" --candidates 6 > $O/bench_c6.json 2> $O/bench_c6.err || exit 1
