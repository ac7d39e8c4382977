# round 3: f32 window store policy (buffer-store aux bits) at 65,536 (output fits the 256 MB
# Infinity Cache) and 131,072 instances (it does not), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03wp; mkdir -p $O
for n in 131072 65536; do
  for v in 16 0 2 17 18; do
    if [ $v = 16 ]; then L=""; else L=$PWD/profiles/_bin/libmz_env_wpol$v.so; fi
    MZ_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py --envs $n --legs window --steps 500 --warmup 50 --train-steps 0 --no-cpu-baseline > $O/wp_${n}_$v.json 2> $O/wp_${n}_$v.err || { tail -20 $O/wp_${n}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/wp_${n}_$v.json')); print($n, $v, round(d['ms_per_step']*1e3,2), round(d['roofline']['frac'],3))"
  done
done
