#!/bin/bash
# round 5: instances per wave of k_step at 65,536 x 81 — 16 (default) vs 4 and 8, window and
# bits legs, interleaved (k_step by HIP events over graph replays)
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in default ipw32 ipw64 default ipw32 ipw64; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 300 python -u bench.py --steps 1000 --warmup 100 --train-steps 0 --curriculum-steps 0 \
    --config-legs "" --no-cpu-baseline > $O/bench_$lib.json 2>> $O/bench.err || exit 1
  python3 -c "
import json;d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]);b=d['bits_mode']
print(json.dumps({'lib':'$lib','window':d['value'],'window_us':d['roofline'].get('avg_kernel_ms',0)*1e3,'bits':b['value'],'bits_us':b['roofline']['avg_kernel_ms']*1e3}))" >> $O/ipw2.jsonl
done
