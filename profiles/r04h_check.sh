set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mcclendon_gpu.py tests/test_gpu_env.py tests/test_bank.py tests/test_checkpoint_gpu.py tests/test_trainer_kernels.py > gpurun_out/r04h/tests.log 2>&1 && \
timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py > gpurun_out/r04h/mc_wg.jsonl 2> gpurun_out/r04h/mc_wg.err && \
timeout -k 10 900 python -u bench.py > gpurun_out/r04h/bench.json 2> gpurun_out/r04h/bench.err
