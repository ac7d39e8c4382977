#!/bin/bash
# round 6: config 5 (PPO, 4,096 toroidal 17..79, fixed sizes) kernel stats at the final sources
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ppo/kt -o run -- python3 bench.py --steps 10 --warmup 2 --legs bits --no-cpu-baseline --train-steps 0 --curriculum-steps 0 --config-legs cfg5 --cfg5-modes fixed --cfg5-steps 600 --cfg-eval-mazes 64 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cp /tmp/ppo/kt/run_kernel_stats.csv $O/ppo_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r06v/ppo_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{float(r["TotalDurationNs"]) / 1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"]) / 1e3:8.1f} us  {r["Name"][:100]}')
print("total ms", tot / 1e6)
PY
