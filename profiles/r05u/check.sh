#!/bin/bash
# round 5: learner launch tails — two-level last-workgroup tickets (k_adamw, k_head_loss) and
# k_colsum over more workgroups: the touched GPU tests, kernel-alone A/B vs HEAD's kernels
# (profiles/_bin/lib_tk1.so = one-level tickets, the old k_colsum), best-of-6 DDQN training A/B
# (interleaved), a kernel trace of the whole training leg (late vector steps), then the whole GPU
# suite and smoke().
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
timeout -k 10 60 ./profiles/_bin/ubench_ticket > $O/ticket.jsonl 2>&1 || exit 1
cat $O/ticket.jsonl
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_flat_optim.py tests/test_head_loss.py tests/test_graph_linear.py tests/test_learner.py \
  tests/test_learner_graph.py tests/test_determinism_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_tk1.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 120 python -u profiles/exp_adamw_ticket.py >> $O/adamw.jsonl || exit 1
  timeout -k 10 120 python -u profiles/exp_head_loss_time.py >> $O/head_loss.jsonl || exit 1
  timeout -k 10 120 python -u profiles/exp_colsum_time.py >> $O/colsum.jsonl || exit 1
done
cat $O/adamw.jsonl $O/head_loss.jsonl $O/colsum.jsonl
for lib in prev new prev new; do
  if [ $lib = prev ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_tk1.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --curriculum-steps 0 \
    --config-legs "" --candidates 6 > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);w=d['win_rate']
print(json.dumps({'lib':'$lib','train_env_steps_per_s':w['train_env_steps_per_s'],'greedy':w['greedy'],'greedy_best_of_6':w['greedy_best_of_6']}))" >> $O/train.jsonl
done
cat $O/train.jsonl
unset MZ_LIB_OVERRIDE
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr/kt -o run -- python3 bench.py --steps 10 --warmup 2 --legs bits --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= --candidates 6 > $O/kt.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 1800 --top 25 > $O/train_streams_late.json || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 50 --top 25 > $O/train_streams_all.json || exit 1
cp /tmp/tr/kt/run_kernel_stats.csv $O/train_kernel_stats.csv
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -3 $O/smoke.log
