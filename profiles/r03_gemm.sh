# round 3: split-precision learner GEMM — tests, then timing vs hipBLASLt f32 (grid targets 256 / 512)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_x3.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 256 512; do
MZ_GEMM_WG_TARGET=$t timeout -k 10 180 python -u profiles/exp_gemm_x3.py > $O/gemm_$t.json 2> $O/gemm_$t.err || { tail -20 $O/gemm_$t.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/gemm_$t.json')); print($t, {k:(v['f32_us'], v['mz_gemm_x3_us']) for k,v in d.items()})"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 profiles/exp_gemm_x3.py > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
grep -E "k_split|k_gemm" $O/kt/run_kernel_stats.csv | cut -c1-140
