#!/bin/bash
# round 6: bench.py's N > 1 path rehearsed on the one GPU — 4 self-launched ranks over gloo
# (MZ_DIST_BACKEND=gloo; the driver's 8-GPU runs use RCCL), every leg at reduced sizes: weak-scaled
# env steps, the sharded-optimizer DDQN leg (+ seen / infer protocols), both curriculum legs (the
# global rule's per-step win all-gather over ranks), configs 1 (rank 0) / 2 / 4 / 5 (the growth
# leg's MIN all-reduce of the retired flags)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06i2
mkdir -p $O
export PYTHONUNBUFFERED=1
MZ_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 4 --envs 16384 --steps 100 --warmup 10 --train-steps 100 --curriculum-steps 100 \
  --curriculum-pi-envs 256 --curriculum-pi-steps 100 --cfg1-episodes 40 \
  --eval-mazes 100 --cfg4-envs 2048 --cfg5-envs 1024 --cfg4-steps 50 --cfg5-steps 50 --cfg-eval-mazes 50 \
  > $O/bench4.json 2> $O/bench4.err || { tail -30 $O/bench4.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench4.json').read().strip().splitlines()[-1])
print({k:d.get(k) for k in ('n_gpus','value','ms_per_step','scaling')}, d.get('config'), list(d.get('configs',{}).keys()))
c=d['curriculum_leg']; print('global', c['total_wins'], c['instances_per_algorithm_at_end'])"
