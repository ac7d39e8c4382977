#!/bin/bash
# round 6: the learner's f32 GEMMs — PyTorch TunableOp (hipBLASLt / rocBLAS solutions timed per
# shape, the fastest kept; tuned once into a results file, then reused) and rocBLAS as the
# preferred library, vs the default hipBLASLt choice: best-of-6 DDQN training leg (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06h
mkdir -p $O
export PYTHONUNBUFFERED=1
ARGS="--steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 --config-legs= --candidates 6"
row() {
  python3 -c "
import json;d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'mode':'$1','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
}
# tuning pass (writes the results file)
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv \
  timeout -k 10 600 python -u bench.py $ARGS > $O/bench_tune.json 2>> $O/bench.err || exit 1
row tune
ls $O
for mode in default tuned default tuned; do
  if [ $mode = tuned ]; then
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv \
      timeout -k 10 400 python -u bench.py $ARGS > $O/bench_$mode.json 2>> $O/bench.err || exit 1
  else
    timeout -k 10 400 python -u bench.py $ARGS > $O/bench_$mode.json 2>> $O/bench.err || exit 1
  fi
  row $mode
done
cat $O/train.jsonl
