set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qact.py tests/test_abi.py > gpurun_out/r04g/tests.log 2>&1 && \
bash profiles/exp_qact_split.sh && \
bash profiles/cfg2_trace.sh gpurun_out/r04f
