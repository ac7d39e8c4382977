#!/bin/bash
# round 6: k_qfc1 as a persistent grid (MZ_QFC1_WGS 256 / 512; 0 = one workgroup per tile in the
# loop wrapper) vs the final library: Q-value checksums, QAct tests, training A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06w
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in final q0 q256 q512; do
  export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qact.py > $O/tests_$lib.log 2>&1 || { tail -20 $O/tests_$lib.log; exit 1; }
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py > $O/checksum_$lib.json 2>> $O/ck.err || exit 1
done
tail -n1 $O/tests_*.log; md5sum $O/checksum_*.json
for lib in final q0 q256 q512 final q0 q256 q512; do
  export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
