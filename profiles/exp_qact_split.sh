# Round 4 (VERDICT next 6): split acting forward (k_qconv + k_qfc1, default) vs the fused k_qact1
# (MZ_QACT_FUSED=1 build): Q checksums, q_head timing alone and the DDQN training leg, interleaved.
set -o pipefail
out=gpurun_out/r04g; mkdir -p $out
for lib in default profiles/_bin/lib_qact_fused.so; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py >> $out/checksum.jsonl || exit 1
done
for rep in 1 2; do
  for lib in default profiles/_bin/lib_qact_fused.so; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs '' --eval-mazes 200 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
