#!/bin/bash
# round 6 final sources: the whole GPU test suite, smoke(), the k_step kernel traces + PMC passes
# (profiles/collect.sh, summarised by profiles/summarize.py), and a kernel trace of the best-of-6
# DDQN training leg reduced to per-stream busy times (profiles/train_streams.py; the raw trace
# stays in /tmp: gpurun_out comes back only under 64 MiB)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06final
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 bash profiles/collect.sh > $O/collect.log 2>&1 || { tail -20 $O/collect.log; exit 1; }
P=gpurun_out/prof
for m in window bits; do
  python3 profiles/summarize.py r06_$m $P/kt_$m $P/fetch_$m $P/write_$m --mode $m > $O/pmc_$m.json || exit 1
  cp profiles/r06_${m}_kernel_stats.csv $O/
done
cp profiles/pmc_k_step.json $O/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr/kt -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= > $O/train_kt.log 2>&1 || { tail -20 $O/train_kt.log; exit 1; }
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 1800 --top 25 > $O/train_streams_late.json || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 50 --top 25 > $O/train_streams_all.json || exit 1
cp /tmp/tr/kt/run_kernel_stats.csv $O/train_kernel_stats.csv
du -sh gpurun_out
# the full default bench (the driver's command at N = 1)
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
