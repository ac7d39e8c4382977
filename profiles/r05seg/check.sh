#!/bin/bash
# round 5: bits-only k_step with the window as 15-bit segments in LDS (plain 2-B stores, words
# assembled at the store) instead of LDS atomics into a zeroed bit string: env GPU tests (window
# bits vs the oracle every step), then both legs A/B vs MZ_BITS_SEG=0 (interleaved, 400 replays)
set -o pipefail
O=gpurun_out/r05seg
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_env.py \
  tests/test_greedy_rows.py tests/test_trainer_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in seg0 new seg0 new seg0 new; do
  if [ $lib = seg0 ]; then export MZ_LIB_OVERRIDE=profiles/_bin/lib_seg0.so; else unset MZ_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u bench.py --steps 400 --warmup 40 --legs window,bits --train-steps 0 --curriculum-steps 0 \
    --config-legs "" --no-cpu-baseline > $O/b_$lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]);b=d['bits_mode'];print(json.dumps({'lib':'$lib','window':d['value'],'window_us':d['roofline']['avg_kernel_ms']*1e3,'bits':b['value'],'bits_us':b['roofline']['avg_kernel_ms']*1e3,'bits_frac':b['roofline']['frac']}))" >> $O/ab.jsonl
done
cat $O/ab.jsonl
