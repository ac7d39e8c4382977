#!/bin/bash
# round 5: k_reset_done ranks a group's winners from k_bank_count's stored codes (the race: with
# several waves per 64-instance group, a wave could read instances a sibling had already reset).
# Per-step fingerprints x3, the determinism test x2, the bank / schedule / env tests.
set -o pipefail
O=gpurun_out/r05z3
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 200 python -u profiles/exp_det_steps.py 450 >> $O/steps.jsonl 2>> $O/steps.err || { tail -20 $O/steps.err; exit 1; }
done
python3 - <<'PY'
import json
names=['greedy','count','actions','reward','obs6','steps_done','eps','algo']
g=[json.loads(l)['rec'] for l in open('gpurun_out/r05z3/steps.jsonl')]
for j in range(1,len(g)):
    a,b=g[0],g[j]; first=None
    for k in range(min(len(a),len(b))):
        d=[names[c] for c in range(8) if a[k][c]!=b[k][c]]
        if d: first=(k,d); break
    print('run0 vs run%d:'%j, first)
PY
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_determinism_gpu.py >> $O/det.log 2>&1 || { tail -30 $O/det.log; exit 1; }
done
grep -E 'passed|failed' $O/det.log
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_bank.py \
  tests/test_best_of_bank.py tests/test_schedule.py tests/test_gpu_env.py tests/test_greedy_rows.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
