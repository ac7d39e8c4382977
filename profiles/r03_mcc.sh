# round 3: GPU McClendon kernel tests + timing, then the full GPU suite and bench (QW1=8 QAct)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_mcclendon_gpu.py tests/test_greedy_rows.py > $O/mcc_tests.log 2>&1 || { tail -60 $O/mcc_tests.log; exit 1; }
tail -3 $O/mcc_tests.log
timeout -k 10 300 python -u profiles/exp_mcclendon.py > $O/mcc_timing.json 2> $O/mcc_timing.err || { tail -20 $O/mcc_timing.err; exit 1; }
cat $O/mcc_timing.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 4000 $O/bench.json
