#!/bin/bash
# round 6: the screen with batched flag / parent passes and a worklist for the root jumping —
# tests, fill A/B vs the previous library, per-step clock stamps (profiling build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06s
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_screen_gpu.py \
  tests/test_best_of_bank.py tests/test_mcclendon_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in lanesrp default lanesrp default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
done
true
python3 - <<'PY'
import json
for l in open("gpurun_out/r06s/fill.jsonl"):
    d = json.loads(l); print(d["lib"], d["algorithm"], d["ms"], d["slots_sha"])
PY
