#!/bin/bash
# round 6: (1) TunableOp tuning pass over every learner GEMM shape the bench's legs use (short legs,
# the default batch sizes) -> the results file to commit, installed for the steps after; (2) the
# Philox-ring lite carves: tests, fill rate and best-of-6 DDQN training vs the previous library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06j
mkdir -p $O
export PYTHONUNBUFFERED=1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv \
  timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --train-steps 60 \
  --curriculum-steps 60 --curriculum-pi-steps 60 --cfg1-episodes 5 --cfg2-steps 60 --cfg4-steps 60 --cfg5-steps 60 \
  --eval-mazes 64 --cfg-eval-mazes 64 > $O/bench_tune.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
wc -l $O/tunableop0.csv
cp $O/tunableop0.csv maze-solving-agent-gymnasium_amd/mazerl/tuning/gemm_gfx950.csv
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_build_algorithms.py \
  tests/test_best_of_bank.py tests/test_screen_gpu.py tests/test_bank.py tests/test_learner.py tests/test_head_loss.py \
  tests/test_determinism_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in r06scr default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
done
cat $O/fill.jsonl
for lib in r06scr default r06scr default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6'],'sel':w.get('training_mazes',{}).get('selection_stats')}))" >> $O/train.jsonl
done
cat $O/train.jsonl
