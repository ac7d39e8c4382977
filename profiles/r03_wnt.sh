# round 3: window store policy chosen by size — env GPU tests, bench at 65,536 and 131,072, then
# the k_step PMC records for the new sources (profiles/collect.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03nt; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_dropin.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 65536 131072; do
  timeout -k 10 300 python -u bench.py --envs $n --train-steps 0 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$n.json')); print($n, round(d['ms_per_step']*1e3,2), round(d['roofline']['frac'],3), round(d['bits_mode']['ms_per_step']*1e3,2))"
done
bash profiles/collect.sh || exit 1
echo collect-ok
