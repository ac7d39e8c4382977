set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_flat_optim.py tests/test_trainer_kernels.py "tests/test_gpu_env.py::test_headline_config_every_lane_autoreset_vs_oracle" "tests/test_gpu_env.py::test_act_draw_follows_reference_exploration_distribution" > $O/new_tests.log 2>&1 || { tail -50 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 3000
