# Round 4: k_adamw with the loads of MZ_ADAMW_U grid-stride iterations issued together and the
# segment base pointers from an LDS table (default U = 4; lib_adamw_u2: U = 2) vs the previous
# commit's k_adamw (lib_adamw_head). The flat-AdamW GPU tests, then training A/B interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04v; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_flat_optim.py tests/test_learner_overlap.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
LIBS="default profiles/_bin/lib_adamw_u2.so profiles/_bin/lib_adamw_head.so"
for rep in 1 2; do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs cfg4 --curriculum-steps 0 --eval-mazes 200 --cfg-eval-mazes 100 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
unset MZ_LIB_OVERRIDE
echo ok
