#!/bin/bash
# round 6: lite dfs candidate regions: tests, fill rate vs the r-prim-only lite library, and a
# kernel trace of the best-of-6 DDQN training leg (per-stream busy time, late vector steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06f
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_screen_gpu.py \
  tests/test_best_of_bank.py tests/test_build_algorithms.py tests/test_bank.py tests/test_schedule.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in r06lite default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_bestof_fill.py 2048 >> $O/fill.jsonl 2>> $O/fill.err || exit 1
done
unset MZ_LIB_OVERRIDE
cat $O/fill.jsonl
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr/kt -o run -- python3 bench.py --steps 10 --warmup 2 --legs bits --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= --candidates 6 > $O/kt.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 1800 --top 25 > $O/train_streams_late.json || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 50 --top 25 > $O/train_streams_all.json || exit 1
cp /tmp/tr/kt/run_kernel_stats.csv $O/train_kernel_stats.csv
head -c 2500 $O/train_streams_late.json
