# Round 4: k_qfc1's workgroup -> XCD mapping: 1 output tile per XCD (default; A chunks of a row tile
# read by 4 XCDs) vs 2 / 4 output tiles per XCD cycled over consecutive workgroups (lib_ntx2 /
# lib_ntx4: A read by 2 / 1 XCDs, 2 / 4 weight slices per L2). Q checksums, training + q_head A/B
# interleaved, one FETCH_SIZE pass per library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04q; mkdir -p $out
LIBS="default profiles/_bin/lib_ntx2.so profiles/_bin/lib_ntx4.so"
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
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES -f csv -d $out/pmc_$b -o run -- python3 profiles/exp_qact.py prof > $out/pmc_$b.log 2>&1 || exit 1
done
unset MZ_LIB_OVERRIDE
echo ok
