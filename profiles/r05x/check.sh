#!/bin/bash
# round 5: (1) head-loss forward / backward kernels alone vs the committed ones (prev), (2) the
# best-of-6 DDQN leg + configs 2 / 4, prev vs new, interleaved, (3) five determinism trails of the
# live run (digest per 25 vector steps, K-update graph on) at the working tree, to find where
# runs part (r05u / r05w: intermittent), (4) the learner GPU tests.
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 120 python -u profiles/exp_head_loss_time.py >> $O/head_loss.jsonl || exit 1
done
cat $O/head_loss.jsonl
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs cfg2,cfg4 --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate'];c=d['configs']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'cfg2':c['cfg2']['env_steps_per_s'],'cfg2_greedy':c['cfg2']['win_rate_greedy'],'cfg4':c['cfg4']['env_steps_per_s'],'cfg4_greedy':c['cfg4']['win_rate_reference_protocol']['greedy']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
unset MZ_LIB_OVERRIDE
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u profiles/exp_det_trail.py 600 >> $O/trail.jsonl 2>> $O/trail.err || { tail -20 $O/trail.err; exit 1; }
done
python3 - <<'PY'
import json
rs=[json.loads(l) for l in open('gpurun_out/r05x/trail.jsonl')]
for r in rs:
    print(r['kblock'], ' '.join(t['r'][:4] for t in r['trail']))
PY
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_head_loss.py tests/test_learner.py tests/test_learner_graph.py tests/test_learner_overlap.py \
  tests/test_trainer_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
