#!/bin/bash
# AdamW step count folded into k_adamw (last-workgroup ticket) + persistent backward seed: the
# optimizer / learner tests, then the training leg of bench.py (twice). Usage: <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_flat_optim.py tests/test_learner_graph.py tests/test_learner_overlap.py tests/test_gpu_distributed.py tests/test_trainer_kernels.py tests/test_learner.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 &&
for f in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done
