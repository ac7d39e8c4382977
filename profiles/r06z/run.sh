#!/bin/bash
# round 6: k_head_loss's 12 row-sum butterflies side by side — learner tests, weight digests vs the
# previous library (bit-identical expected), update timing at batch 512 / 1,024
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06z
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_determinism_gpu.py \
  tests/test_head_loss.py tests/test_learner.py tests/test_learner_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in prevhl default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python3 profiles/exp_learner_digest.py >> $O/digest.jsonl || exit 1
done
cat $O/digest.jsonl
for lib in prevhl default prevhl default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  for b in 512 1024; do
    timeout -k 10 200 python3 profiles/exp_update_kernels.py $b | sed "s/}/, \"lib\": \"$lib\"}/" >> $O/update.jsonl || exit 1
  done
done
cat $O/update.jsonl
