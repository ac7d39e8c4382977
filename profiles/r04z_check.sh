# Round 4: k_reset_done's rare in-place build moved out of line with the handle by value (every
# wave copied the 376-B MzDev kernel argument to scratch on entry) — the reset / bank / checkpoint
# GPU tests, training A/B vs the previous mz_env.hip (lib_env_head), then the k_step kernel trace
# and PMC passes at the new sources (profiles/collect.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04z; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py tests/test_trainer_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
LIBS="default profiles/_bin/lib_env_head.so"
for rep in 1 2; do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs cfg4 --curriculum-steps 0 --eval-mazes 200 --cfg-eval-mazes 100 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
unset MZ_LIB_OVERRIDE
bash profiles/collect.sh || { echo "collect failed"; exit 1; }
for leg in window bits; do tail -2 gpurun_out/prof/kt_$leg.log; done
du -sh gpurun_out/prof
