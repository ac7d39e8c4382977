# Round 4: trace of config 4's training leg (8,192 mixed 81x81 DDQN, 4 updates of 512 per vector
# step) for the per-stream breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --legs bits --steps 10 --warmup 2 --train-steps 0 --curriculum-steps 0 --no-cpu-baseline --config-legs cfg4 --cfg4-steps 300 --cfg-eval-mazes 32 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python3 profiles/train_streams.py $O/kt/run_kernel_trace.csv --skip 50 --top 25 --step-kernel "k_step<4, false, true, true, false>" > $O/cfg4_train_streams.json || { grep -o "k_step<[^>]*>" $O/kt/run_kernel_trace.csv | sort | uniq -c; exit 1; }
cp $O/kt/run_kernel_stats.csv $O/cfg4_kernel_stats.csv; rm -rf $O/kt
