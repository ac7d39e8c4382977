set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/snap
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_learner_overlap.py tests/test_head_kernels.py tests/test_greedy_rows.py tests/test_learner_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for V in new full new full; do
  if [ $V = full ]; then export MZ_AB_FULL_SNAPSHOT=1; else unset MZ_AB_FULL_SNAPSHOT; fi
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$V.json
  python3 -c "import json,sys; d=json.load(open('$O/bench_$V.json')); w=d['win_rate']; print(json.dumps({'snapshot': '$V', 'train_env_steps_per_s': w['train_env_steps_per_s'], 'greedy': w['greedy'], 'greedy_best_of_6': w['greedy_best_of_6']}))" >> $O/train.jsonl
done
