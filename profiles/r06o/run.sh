#!/bin/bash
# round 6: lane-parallel lite carves (mz_lite_carve_lanes) — tests, then the fill rate and slot
# hashes vs the ring library (profiles/_bin/lib_r06ring.so) and 8 / 16 mazes per wave, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06o
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_build_algorithms.py \
  tests/test_best_of_bank.py tests/test_screen_gpu.py tests/test_bank.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in r06ring default lanes8 lanes16 r06ring default lanes8 lanes16; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06o/fill.jsonl"):
    d = json.loads(l); print(d["lib"], d["algorithm"], d["ms"], d["slots_sha"])
PY
