# Round 4: the overlapped learner's K updates per vector step as one graph replay (MZ_K_BLOCK=1,
# default) vs K single-update replays (MZ_K_BLOCK=0): the equivalence GPU test, then config 4 and
# the curriculum leg (both 4 updates per vector step) A/B interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04zz; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_learner_overlap.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for kb in 1 0; do
    MZ_K_BLOCK=$kb timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --train-steps 0 --config-legs cfg4 --curriculum-steps 1200 --eval-mazes 200 --cfg-eval-mazes 100 > $out/bench_${rep}_kb$kb.json 2>> $out/bench.err || exit 1
  done
done
echo ok
