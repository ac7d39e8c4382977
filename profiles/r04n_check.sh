# Round 4: the split acting forward at 8 waves per workgroup (k_qfc1 64 rows x 512 outputs: each A
# tile read by 2 output tiles instead of 4; k_qconv 2 conv tiles per wave) vs 4, interleaved;
# then the 4-rank gloo rehearsal of the whole bench through its own launcher
set -o pipefail
out=gpurun_out/r04n; mkdir -p $out
for lib in default profiles/_bin/lib_qw8.so profiles/_bin/lib_qb2.so; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py >> $out/checksum.jsonl || exit 1
done
for rep in 1 2; do
  for lib in default profiles/_bin/lib_qw8.so profiles/_bin/lib_qb2.so; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs cfg4 --curriculum-steps 0 --eval-mazes 200 --cfg-eval-mazes 100 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
unset MZ_LIB_OVERRIDE
MZ_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench.py --gpus 4 --envs 16384 --cfg4-envs 2048 --cfg5-envs 1024 --curriculum-envs 1024 --curriculum-steps 600 --eval-mazes 300 --cfg-eval-mazes 200 > $out/bench4.json 2> $out/bench4.err
