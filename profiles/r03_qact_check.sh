set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_qact.py tests/test_greedy_rows.py tests/test_learner_overlap.py tests/test_learner_graph.py tests/test_qfront.py tests/test_trainer_kernels.py > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" $O/tests.log | head -60
exit $rc
