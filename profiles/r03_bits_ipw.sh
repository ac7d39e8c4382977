# round 3: bits-mode k_step at 65,536 x 81x81 with 16 vs 4 instances per wave (interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03s; mkdir -p $O
B="--legs bits --steps 1000 --warmup 100 --no-cpu-baseline --train-steps 0"
for r in 1 2; do
  for v in 16 32; do
    MZ_STEP_BITS_IPW=$v timeout -k 10 200 python -u bench.py $B > $O/ipw_${v}_$r.json 2> $O/ipw_${v}_$r.err || { tail -20 $O/ipw_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ipw_${v}_$r.json')); print($v, d['ms_per_step']*1e3, d['roofline']['frac'])"
  done
done
