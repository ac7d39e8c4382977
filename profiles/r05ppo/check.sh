#!/bin/bash
# round 5: where config 5 (PPO, 4,096 toroidal 17..79) spends its time now: rocprofv3 kernel
# stats of the bench's cfg5 leg (600 vector steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ppo
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ppo/kt -o run -- python3 bench.py --steps 10 --warmup 2 \
  --legs bits --train-steps 0 --curriculum-steps 0 --no-cpu-baseline --config-legs cfg5 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cp /tmp/ppo/kt/run_kernel_stats.csv $O/ppo_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r05ppo/ppo_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:30]:
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['TotalDurationNs'])/1e6,1), round(100*float(r['TotalDurationNs'])/tot,1))
PY
