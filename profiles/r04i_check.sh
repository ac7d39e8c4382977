set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 300 python -u profiles/exp_bestdir_policy.py > gpurun_out/r04i/bestdir.json 2> gpurun_out/r04i/bestdir.err && \
timeout -k 10 400 python -u bench.py --legs bits --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --config-legs '' > gpurun_out/r04i/curr_2400.json 2> gpurun_out/r04i/curr.err && \
timeout -k 10 400 python -u bench.py --legs bits --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --config-legs '' --curriculum-steps 9600 > gpurun_out/r04i/curr_9600.json 2>> gpurun_out/r04i/curr.err
