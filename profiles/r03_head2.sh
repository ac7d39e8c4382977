# round 3 final HEAD check: every GPU test, smoke, the default bench line, rocprofv3 kernel stats
# of the bench (k_step / k_build averages), a training trace's per-stream breakdown, a 2-rank gloo
# rehearsal of bench.py's N>1 path (both ranks on this GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN_TAG:-r03zz}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['win_rate']['train_env_steps_per_s'], d['win_rate']['greedy'], d['win_rate']['greedy_best_of_6'], d['generation']['steady_mazes_per_s'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o bench -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --train-steps 1200 --eval-mazes 64 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
for f in $(find $O/prof -name '*kernel_stats.csv'); do cp $f $O/kernel_stats.csv; done
for f in $(find $O/prof -name '*kernel_trace.csv'); do python3 profiles/train_streams.py $f > $O/train_streams.json; rm -f $f; done
MZ_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --envs 16384 --steps 100 --warmup 10 --train-steps 60 --eval-mazes 100 > $O/rehearsal_2rank.txt 2>&1 || { tail -30 $O/rehearsal_2rank.txt; exit 1; }
tail -c 600 $O/rehearsal_2rank.txt
