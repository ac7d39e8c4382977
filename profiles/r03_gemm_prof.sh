set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_gemm_x3.py > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
grep -E "k_split|k_gemm" $O/kt/run_kernel_stats.csv | cut -c1-160
