# round 3: config-5 PPO vector step under rocprofv3 (kernel trace + stats): where the update's
# 36 ms and the reset / regeneration's 0.6 ms per vector step go
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o; mkdir -p $O
true
true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/ppo_breakdown.py > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
head -25 $O/kt/run_kernel_stats.csv | cut -c1-220
timeout -k 10 180 python -u profiles/exp_gemm_x3.py > $O/gemm_x3.json 2> $O/gemm_x3.err || { tail -20 $O/gemm_x3.err; exit 1; }
cat $O/gemm_x3.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_greedy_rows.py > $O/greedy_rows_tests.log 2>&1 || { tail -40 $O/greedy_rows_tests.log; exit 1; }
tail -3 $O/greedy_rows_tests.log
