#!/bin/bash
# round 6: resident cap of the bank refill's candidate builds (MZ_BANK_WGS: 768 / 1280 / 1792
# workgroups vs the default 4096-workgroup grid) in best-of-6 DDQN training, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06t2
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in wgs1280 wgs1024 wgs1536 wgs1280s768 wgs1280s1024 wgs1280 wgs1024 wgs1536 wgs1280s768 wgs1280s1024; do
  export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
