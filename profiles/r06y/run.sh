#!/bin/bash
# round 6: the learner's shared dropout counter advanced by the source stem's backward
# (MZ_STEM_COUNTER_FOLD=1, default) vs an add launch per forward (=0): learner GPU tests, the
# update alone at batch 512 / 1,024, config 4 and the training leg, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06y
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_checkpoint_gpu.py \
  tests/test_determinism_gpu.py tests/test_gpu_distributed.py tests/test_head_loss.py tests/test_learner.py \
  tests/test_learner_graph.py tests/test_learner_overlap.py tests/test_stem.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 1 0 1; do
  for b in 512 1024; do
    MZ_STEM_COUNTER_FOLD=$f timeout -k 10 200 python3 profiles/exp_update_kernels.py $b | sed "s/}/, \"fold\": $f}/" >> $O/update.jsonl || exit 1
  done
done
cat $O/update.jsonl
for f in 0 1 0 1; do
  MZ_STEM_COUNTER_FOLD=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs cfg4 --cfg4-steps 3000 --cfg-eval-mazes 50 > $O/bench_$f.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]);w=d['win_rate'];c=d['configs']['cfg4']
print(json.dumps({'fold':$f,'train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'cfg4':c['env_steps_per_s']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
