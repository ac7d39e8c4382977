set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mcclendon_gpu.py tests/test_greedy_rows.py > gpurun_out/r04b/tests.log 2>&1 && \
timeout -k 10 300 python -u profiles/exp_mcclendon.py > gpurun_out/r04b/mcclendon_timing.json 2> gpurun_out/r04b/mcclendon_timing.err
