#!/bin/bash
# round 5: test_determinism_gpu failed in r05u (two K single-update runs differed). Trails of the
# live run (digest per 50 vector steps) twice for HEAD's package (profiles/_bin/headwt) and twice
# for the working tree (k_colsum change), MZ_K_BLOCK=0; then the determinism test itself.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export PYTHONUNBUFFERED=1 MZ_K_BLOCK=0
for pkg in head cur head cur; do
  if [ $pkg = head ]; then export MZ_PKG_ROOT=profiles/_bin/headwt; else unset MZ_PKG_ROOT; fi
  timeout -k 10 200 python -u profiles/exp_det_trail.py 600 >> $O/trail.jsonl 2>> $O/trail.err || { tail -20 $O/trail.err; exit 1; }
done
python3 - <<'PY'
import json
rs=[json.loads(l) for l in open('gpurun_out/r05v/trail.jsonl')]
for r in rs:
    print(r['pkg'], r['kblock'], ' '.join(t['src'][:6]+'/'+t['r'][:4] for t in r['trail']))
PY
unset MZ_PKG_ROOT MZ_K_BLOCK
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_determinism_gpu.py > $O/det.log 2>&1; tail -3 $O/det.log
