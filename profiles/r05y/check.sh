#!/bin/bash
# round 5: the live run parts between vector steps 375 and 400 in 4 of 5 runs (r05x). Which
# feature carries the race: three runs each with the overlapped learner off, the maze bank off,
# the curriculum off, and as is.
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export PYTHONUNBUFFERED=1
run() { timeout -k 10 200 python -u profiles/exp_det_trail.py 450 >> $O/trail.jsonl 2>> $O/trail.err || { tail -20 $O/trail.err; exit 1; }; }
for i in 1 2 3; do
  MZ_TRAIL_BANK=0 run
  MZ_TRAIL_CURR= run
  MZ_TRAIL_OVERLAP=0 run
  run
done
python3 - <<'PY'
import json
rs=[json.loads(l) for l in open('gpurun_out/r05y/trail.jsonl')]
for r in sorted(rs, key=lambda r: json.dumps(r['variant'], sort_keys=True)):
    print(json.dumps(r['variant'], sort_keys=True), ' '.join(t['r'][:4] for t in r['trail'][10:]))
PY
