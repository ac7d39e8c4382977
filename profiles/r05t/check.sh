#!/bin/bash
# round 5 (re-entry): the GPU suite + smoke at HEAD, and the last-workgroup ticket microbenchmark
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./profiles/_bin/ubench_ticket > $O/ticket.jsonl 2>&1 || exit 1
cat $O/ticket.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -5 $O/smoke.log
