#!/bin/bash
# round 6: best-of-6 fill A/B (round-5 library vs the screen pipeline), the fill's kernel mix, and the
# best-of-6 DDQN training leg A/B (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06b
mkdir -p $O
export PYTHONUNBUFFERED=1
PREV=profiles/_bin/lib_r05.so
MZ_LIB_OVERRIDE=$PREV timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
cat $O/fill.jsonl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fill -- python3 profiles/exp_bestof_fill.py 2048 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/fill_kernel_stats.csv
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=$PREV; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6'],'sel':w.get('training_mazes',{}).get('selection_stats')}))" >> $O/train.jsonl
done
cat $O/train.jsonl
