# Round 4: GPU test suite at the new k_qfc1, then the DDQN training trace (300 vector steps) reduced
# to the per-stream breakdown (profiles/train_streams.py) and kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash profiles/train_trace.sh || { echo "train trace failed"; tail -20 gpurun_out/trace/kt.log; exit 1; }
python3 profiles/train_streams.py gpurun_out/trace/kt/run_kernel_trace.csv --skip 50 > $O/train_streams.json || exit 1
cp gpurun_out/trace/kt/run_kernel_stats.csv $O/train_kernel_stats.csv; rm -rf gpurun_out/trace
