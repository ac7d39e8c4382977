# Round 4: k_qact2 with 2 chunks per LDS stage (one barrier per 2 chunks, fc2 fragments two chunks
# ahead; lib_q2cpb2) vs 1 (default). Q checksums, training + q_head A/B interleaved, one PMC pass
# per library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04t; mkdir -p $out
LIBS="default profiles/_bin/lib_q2cpb2.so"
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
for lib in $LIBS; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  b=$(basename $lib)
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -f csv -d $out/pmc_$b -o run -- python3 profiles/exp_qact.py prof > $out/pmc_$b.log 2>&1 || exit 1
done
unset MZ_LIB_OVERRIDE
echo ok
