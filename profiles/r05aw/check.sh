#!/bin/bash
# round 5: k_adamw without its last-workgroup ticket (a one-thread launch behind it publishes the
# step count): optimizer / learner / determinism tests, k_adamw alone and the training legs
# (DDQN best-of-6, configs 2 / 4) vs the committed library, interleaved
set -o pipefail
O=gpurun_out/r05aw
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_flat_optim.py \
  tests/test_learner.py tests/test_learner_graph.py tests/test_learner_overlap.py tests/test_determinism_gpu.py \
  tests/test_checkpoint_gpu.py tests/test_gpu_distributed.py tests/test_ppo_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 120 python -u profiles/exp_adamw_ticket.py >> $O/adamw.jsonl || exit 1
done
cat $O/adamw.jsonl
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_prev.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs cfg2,cfg4 --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate'];c=d['configs']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'cfg2':c['cfg2']['env_steps_per_s'],'cfg2_greedy':c['cfg2']['win_rate_greedy'],'cfg4':c['cfg4']['env_steps_per_s'],'cfg4_greedy':c['cfg4']['win_rate_reference_protocol']['greedy']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
