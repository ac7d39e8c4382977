# round 3: the bf16x3 acting head (QAct) — GPU tests, full bench line, training-leg kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench-ok
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --legs bits --train-steps 600 --eval-mazes 200 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo trace-ok
