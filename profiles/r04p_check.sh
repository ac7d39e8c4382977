# Round 4: k_qfc1 / k_qact2 prefetch that actually runs ahead — staging registers as native vectors
# (HIP uint4 / float4 arrays were moved to LDS by promote-alloca: each prefetch waited vmcnt(0)),
# unconditional clamped loads and a prologue in the loop's load order (the s_waitcnt counts), k_qact2
# two chunks ahead, swizzled conflict-free LDS A tiles. Libraries: default (all), lib_swz0 (padded
# 80-B rows), lib_q2a1 (k_qact2's previous loop), lib_head (the previous commit). Q checksums,
# training + q_head A/B interleaved, one PMC pass of LDS / wait counters for default and head.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04p; mkdir -p $out
LIBS="default profiles/_bin/lib_swz0.so profiles/_bin/lib_q2a1.so profiles/_bin/lib_head.so"
for lib in $LIBS; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py >> $out/checksum.jsonl || exit 1
done
for rep in 1 2; do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs cfg4 --curriculum-steps 0 --eval-mazes 200 --cfg-eval-mazes 100 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
for lib in default profiles/_bin/lib_head.so; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  b=$(basename $lib)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -f csv -d $out/pmc_$b -o run -- python3 profiles/exp_qact.py prof > $out/pmc_$b.log 2>&1 || exit 1
done
unset MZ_LIB_OVERRIDE
echo ok
