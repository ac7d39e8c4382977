#!/bin/bash
# round 5: per-vector-step device fingerprints of the live run (overlap + bank + per-instance
# curriculum), four runs: the first step and quantity at which they part
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3 4; do
  timeout -k 10 200 python -u profiles/exp_det_steps.py 450 >> $O/steps.jsonl 2>> $O/steps.err || { tail -20 $O/steps.err; exit 1; }
done
python3 - <<'PY'
import json
rs=[json.loads(l)['rec'] for l in open('gpurun_out/r05z/steps.jsonl')]
names=['greedy','count','actions','reward','obs6','steps_done','eps','algo']
for j in range(1,len(rs)):
    a,b=rs[0],rs[j]
    first=None
    for k in range(min(len(a),len(b))):
        d=[names[c] for c in range(8) if a[k][c]!=b[k][c]]
        if d: first=(k,d); break
    print('run0 vs run%d: first difference at step'%j, first)
PY
