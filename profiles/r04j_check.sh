# Round 4 profile run: k_step kernel stats + PMC (collect.sh), the DDQN training trace's per-stream
# breakdown, config 2's trace after the k_reset_done change, QAct PMC — big CSVs reduced on the box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh || { echo "collect failed"; exit 1; }
for leg in window bits; do tail -3 gpurun_out/prof/kt_$leg.log; done
bash profiles/train_trace.sh || { echo "train trace failed"; tail -20 gpurun_out/trace/kt.log; exit 1; }
python3 profiles/train_streams.py gpurun_out/trace/kt/run_kernel_trace.csv --skip 50 > gpurun_out/trace/train_streams.json || exit 1
cp gpurun_out/trace/kt/run_kernel_stats.csv gpurun_out/trace/train_kernel_stats.csv; rm -rf gpurun_out/trace/kt
bash profiles/cfg2_trace2.sh gpurun_out/r04j || { echo "cfg2 failed"; tail -20 gpurun_out/r04j/kt.log; exit 1; }
python3 profiles/train_streams.py gpurun_out/r04j/kt/run_kernel_trace.csv --skip 50 --step-kernel "k_step<4, false, true, true, false>" > gpurun_out/r04j/cfg2_train_streams.json || exit 1
rm -rf gpurun_out/r04j/kt
bash profiles/r04_qact_pmc.sh || exit 1
du -sh gpurun_out/*
