#!/bin/bash
# round 5: (1) flat gradients + the learner tests; live-trainer determinism, K single-update
# replays vs the K-update graph; (2) k_qconv without the patch LUT: Q-value checksum against the
# round-4 library, timing interleaved, PMC
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_flat_optim.py tests/test_learner.py tests/test_learner_graph.py tests/test_learner_overlap.py \
  tests/test_gpu_distributed.py tests/test_checkpoint_gpu.py tests/test_qact.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread \
  tests/test_determinism_gpu.py > $O/tests_det.log 2>&1
echo "det rc=$?" >> $O/tests_det.log
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_qact_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py > $O/checksum_$lib.json || exit 1
  timeout -k 10 200 python -u profiles/exp_qact.py $lib >> $O/qact_timing.jsonl || exit 1
done
unset MZ_LIB_OVERRIDE
cd /tmp && export TMPDIR=/tmp && cd "$R"
Q=/tmp/qpmc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $Q/kt -o run -- python3 profiles/exp_qact.py prof > $O/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $Q/a -o run -- python3 profiles/exp_qact.py prof > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE -f csv -d $Q/b -o run -- python3 profiles/exp_qact.py prof > $O/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $Q/fetch -o run -- python3 profiles/exp_qact.py prof > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $Q/write -o run -- python3 profiles/exp_qact.py prof > $O/write.log 2>&1 || exit 1
python3 profiles/summarize_qact_pmc.py $Q > $O/qact_pmc.json
# (3) bits-mode k_step: instances per wave (MZ_IPW) variants, interleaved
for lib in default ipw8 ipw32 ipw64 default ipw32 ipw64; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 --legs bits --train-steps 0 --curriculum-steps 0 \
    --config-legs "" --no-cpu-baseline > $O/bits_$lib.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.loads(open('$O/bits_$lib.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'$lib','value':d['value'],'ms':d['ms_per_step'],'kernel_ms':d['roofline']['avg_kernel_ms']}))" >> $O/bits_ipw.jsonl
done
unset MZ_LIB_OVERRIDE
