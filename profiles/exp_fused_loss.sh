#!/bin/bash
# Fused Q-loss: its GPU tests, the learner tests it runs under, then an A/B of bench.py's
# training leg (FUSED_LOSS on / off via MZ_FUSED_LOSS). Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_trainer_kernels.py tests/test_learner_overlap.py tests/test_learner_graph.py tests/test_learner.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for f in 1 0 1 0; do
  MZ_FUSED_LOSS=$f timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"fused_loss\": $f, /" >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
