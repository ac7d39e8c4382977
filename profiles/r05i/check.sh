#!/bin/bash
# round 5, A/Bs against single-file variants of the current library (profiles/build_variant.sh),
# interleaved, each with an output checksum: (1) McClendon phase G lane path vs the wave-only
# phase G; (2) Philox maze builds with the RNG word picked by selects vs the scratch-indexed buffer;
# (3) QAct: round-4 k_qconv (patch rows 17 + LUT), rows 20 without LUT, + MFMA results in VGPRs and
# k_qact_prep1 over 256 workgroups; PMC of the current QAct; (4) k_adamw with batched loads;
# (5) the bench's training leg with best-of-6 training mazes
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_mc_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc_ab.jsonl || exit 1
done
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_gen_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 200 python -u profiles/gen_rate.py --philox-81 >> $O/gen_ab.jsonl || exit 1
done
for lib in old pr20 new new pr20; do
  case $lib in old) export MZ_LIB_OVERRIDE=profiles/_bin/lib_qact_old.so;;
    pr20) export MZ_LIB_OVERRIDE=profiles/_bin/lib_qact_pr20.so;; *) unset MZ_LIB_OVERRIDE;; esac
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py > $O/qact_checksum_$lib.json || exit 1
  timeout -k 10 200 python -u profiles/exp_qact.py $lib >> $O/qact_timing.jsonl || exit 1
done
for lib in old new old new; do
  if [ $lib = old ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_adamw_old.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 120 python -u profiles/exp_adamw_ticket.py >> $O/adamw_ab.jsonl || exit 1
done
unset MZ_LIB_OVERRIDE
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --curriculum-steps 0 \
  --config-legs "" --candidates 6 > $O/bench_c6.json 2> $O/bench_c6.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
Q=/tmp/qpmc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $Q/kt -o run -- python3 profiles/exp_qact.py prof > $O/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $Q/a -o run -- python3 profiles/exp_qact.py prof > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE -f csv -d $Q/b -o run -- python3 profiles/exp_qact.py prof > $O/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $Q/fetch -o run -- python3 profiles/exp_qact.py prof > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $Q/write -o run -- python3 profiles/exp_qact.py prof > $O/write.log 2>&1 || exit 1
python3 profiles/summarize_qact_pmc.py $Q > $O/qact_pmc.json
