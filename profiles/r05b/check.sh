#!/bin/bash
# round 5: where k_mcclendon's time goes (MZ_MC_PROBE variants: the kernel returns after phase k,
# timing only) and a kernel trace of the DDQN win-rate leg with best-of-6 training mazes
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in default 1 2 3 4 5 6 7 default; do
  if [ "$lib" = default ]; then
    timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_probes.jsonl || exit 1
  else
    MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp$lib.so timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_probes.jsonl || exit 1
  fi
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/r05b_prof -o train -- \
  python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --curriculum-steps 0 --config-legs "" \
  --train-steps 600 --eval-mazes 50 --legs bits > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?
find /tmp/r05b_prof -name "*kernel_stats.csv" -exec cp {} $O/ \;
exit $rc
