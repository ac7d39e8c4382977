#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r06y
timeout -k 10 300 python -u profiles/dbg_counter_fold.py 2>&1 | grep -v Warning | tee gpurun_out/r06y/dbg.log
