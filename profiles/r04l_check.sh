# Round 4: QAct after counter-based dropout draws + chunk-group k_qconv; k_qfc1 A-path modes A/B
set -o pipefail
out=gpurun_out/r04l; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_qact.py > $out/tests.log 2>&1 || exit 1
for lib in default profiles/_bin/lib_qact_fused.so profiles/_bin/lib_qfc1_m1.so profiles/_bin/lib_qfc1_m2.so; do
  if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
  timeout -k 10 200 python -u profiles/exp_qact_checksum.py >> $out/checksum.jsonl || exit 1
done
for rep in 1 2; do
  for lib in default profiles/_bin/lib_qfc1_m1.so profiles/_bin/lib_qfc1_m2.so; do
    if [ "$lib" = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$lib; fi
    timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --config-legs= --curriculum-steps 0 --eval-mazes 200 > $out/bench_${rep}_$(basename $lib).json 2>> $out/bench.err || exit 1
  done
done
unset MZ_LIB_OVERRIDE
export PYTHONPATH=$PWD/maze-solving-agent-gymnasium_amd
timeout -k 10 300 python -u bench.py --legs bits --steps 50 --warmup 5 --no-cpu-baseline --train-steps 0 --config-legs cfg4 --curriculum-steps 0 --cfg-eval-mazes 200 > $out/bench_cfg4.json 2>> $out/bench.err || exit 1
timeout -k 10 240 python -u -m mazerl.train --envs 4096 --dim 15 --variant dqn --steps 1600 --batch 2048 --updates-per-step 1 --log-every 0 | tail -1 >> $out/cfg2.jsonl
