#!/bin/bash
# round 5: per-step fingerprints, the maze bank's refills on the main stream vs on their side
# stream (three runs each): is the concurrency of the refills the race?
set -o pipefail
O=gpurun_out/r05z2
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  MZ_TRAIL_BANK_MAIN=1 timeout -k 10 200 python -u profiles/exp_det_steps.py 450 >> $O/steps.jsonl 2>> $O/steps.err || { tail -20 $O/steps.err; exit 1; }
  timeout -k 10 200 python -u profiles/exp_det_steps.py 450 >> $O/steps.jsonl 2>> $O/steps.err || { tail -20 $O/steps.err; exit 1; }
done
python3 - <<'PY'
import json
names=['greedy','count','actions','reward','obs6','steps_done','eps','algo']
rs=[json.loads(l) for l in open('gpurun_out/r05z2/steps.jsonl')]
for mode in ('1', None):
    g=[r['rec'] for r in rs if r['bank_main']==mode]
    for j in range(1,len(g)):
        a,b=g[0],g[j]; first=None
        for k in range(min(len(a),len(b))):
            d=[names[c] for c in range(8) if a[k][c]!=b[k][c]]
            if d: first=(k,d); break
        print('bank_main', mode, 'run0 vs run%d:'%j, first)
PY
