set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_bank.py tests/test_greedy_rows.py tests/test_checkpoint_gpu.py > gpurun_out/r04a/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --train-steps 300 --eval-mazes 200 --cfg-eval-mazes 100 --cfg4-steps 200 --cfg5-steps 200 --no-cpu-baseline > gpurun_out/r04a/bench1.json 2> gpurun_out/r04a/bench1.err && \
MZ_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 4 --envs 16384 --steps 100 --warmup 10 --train-steps 100 --eval-mazes 100 --cfg4-envs 2048 --cfg5-envs 1024 --cfg4-steps 50 --cfg5-steps 50 --cfg-eval-mazes 50 > gpurun_out/r04a/bench4.json 2> gpurun_out/r04a/bench4.err
