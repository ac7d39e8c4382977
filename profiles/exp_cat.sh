#!/bin/bash
# Window-bit assembly without LDS atomics: env parity tests, smoke, then k_step A/B (steady state).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_dropin.py tests/test_qfront.py tests/test_greedy_rows.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
for v in cat_atomic cat_slots cat_atomic cat_slots; do
  timeout -k 10 120 python3 profiles/exp_autoreset.py --lib profiles/_bin/$v.so --warmup 300 --iters 1000 | sed "s/^{/{\"variant\": \"$v\", /" >> $out/ab.jsonl || exit 1
done
for v in cat_atomic cat_slots; do
  timeout -k 10 120 python3 profiles/exp_autoreset.py --lib profiles/_bin/$v.so --toroidal-variable --warmup 300 --iters 1000 | sed "s/^{/{\"variant\": \"$v tor-var\", /" >> $out/ab.jsonl || exit 1
done
