#!/bin/bash
# round 5: k_mcclendon with its resident workgroups capped (MZ_MC_WGS 128 / 256: a persistent
# grid scoring several candidates per workgroup) so that the refills leave CUs' LDS to the
# trainer's kernels: McClendon tests on the capped build, scoring time alone, best-of-6 DDQN
# training vs the uncapped default (interleaved)
set -o pipefail
O=gpurun_out/r05mc
mkdir -p $O
export PYTHONUNBUFFERED=1
MZ_LIB_OVERRIDE=profiles/_bin/lib_mc128.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_mcclendon_gpu.py tests/test_best_of_bank.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in default mc128 mc256; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 300 python -u profiles/exp_mcclendon_wg.py >> $O/mc.jsonl || exit 1
done
for lib in default mc128 mc256 default mc128 mc256; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
