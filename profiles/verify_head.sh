#!/bin/bash
# Round check at HEAD on the GPU box (repo root): GPU test suite, smoke(), default bench line.
# Usage: profiles/verify_head.sh <tag>   -> gpurun_out/<tag>/{gpu_tests.log,smoke.log,bench.json}
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
