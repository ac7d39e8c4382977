#!/bin/bash
# round 5: (1) the fused Q head + loss (tests vs the unfused path, the learner suites); (2) the
# K-update graph in the live trainer (round-4 package twice, current twice, MZ_K_BLOCK=1);
# (3) training traces (DDQN headline leg, config 4) -> per-stream breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_head_loss.py tests/test_learner.py tests/test_learner_graph.py tests/test_learner_overlap.py \
  > $O/tests.log 2>&1 || exit 1
for pkg in old old new new; do
  MZ_K_BLOCK=1 timeout -k 10 400 python -u profiles/r05f/kblock_repro.py $pkg >> $O/kblock.jsonl 2>> $O/kblock.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr/kt -o run -- python3 bench.py --steps 10 --warmup 2 --train-steps 300 --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= > $O/kt.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 50 --top 25 > $O/train_streams.json || exit 1
cp /tmp/tr/kt/run_kernel_stats.csv $O/train_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr4/kt -o run -- python3 bench.py --legs bits --steps 10 --warmup 2 --train-steps 0 --curriculum-steps 0 --no-cpu-baseline --config-legs cfg4 --cfg4-steps 300 --cfg-eval-mazes 32 > $O/kt4.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr4/kt/run_kernel_trace.csv --skip 50 --top 25 --step-kernel "k_step<4, false, true, true, false>" > $O/cfg4_train_streams.json || exit 1
cp /tmp/tr4/kt/run_kernel_stats.csv $O/cfg4_kernel_stats.csv
