#!/bin/bash
# round 5: the K-update graph with persistent index buffers — (1) the determinism test (K single-
# update replays twice, the K-update graph twice, all equal, across train() calls) and the fixed-
# replay bit-equality test; (2) the round-4 curriculum leg's repro with a digest trail, MZ_K_BLOCK
# 0 / 1 / 1; (3) what the K-update graph gains: the curriculum leg (per-instance rule, 4 updates of
# 1,024) and config 4 (4 of 512), MZ_K_BLOCK 0 / 1 interleaved
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_determinism_gpu.py tests/test_learner_overlap.py > $O/tests.log 2>&1 || exit 1
for kb in 0 1 1; do
  MZ_K_BLOCK=$kb timeout -k 10 400 python -u profiles/r05f/kblock_repro.py new >> $O/kblock.jsonl 2>> $O/kblock.err || exit 1
done
for kb in 0 1 0 1; do
  MZ_K_BLOCK=$kb timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --train-steps 0 --no-cpu-baseline \
    --curriculum-rules per-instance --config-legs cfg4 --candidates 1 > $O/bench_kb$kb.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_kb$kb.json').read().strip().splitlines()[-1])
c=d.get('curriculum_leg_per_instance') or d.get('curriculum_leg') or {}
print(json.dumps({'k_block':$kb,'curriculum_env_steps_per_s':c.get('train_env_steps_per_s'),'curriculum_greedy':c.get('greedy'),'cfg4_env_steps_per_s':d['configs']['cfg4']['env_steps_per_s'],'cfg4_greedy':d['configs']['cfg4']['win_rate_reference_protocol']['greedy']}))" >> $O/kblock_gain.jsonl
done
