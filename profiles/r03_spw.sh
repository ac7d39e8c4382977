# round 3: k_step waves per workgroup (MZ_SPW 1 / 2 / 4) in both bench legs, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03sp; mkdir -p $O
B="--legs window,bits --steps 1000 --warmup 100 --no-cpu-baseline --train-steps 0"
for r in 1 2; do
  for v in 1 2 4; do
    if [ $v = 1 ]; then L=""; else L=$PWD/profiles/_bin/libmz_env_spw$v.so; fi
    MZ_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py $B > $O/spw_${v}_$r.json 2> $O/spw_${v}_$r.err || { tail -20 $O/spw_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/spw_${v}_$r.json')); print($v, round(d['ms_per_step']*1e3,2), round(d['bits_mode']['ms_per_step']*1e3,2))"
  done
done
