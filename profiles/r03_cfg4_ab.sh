# round 3: config 4 (per-GPU share: 8,192 x 81x81 mixed, DDQN, 4 updates of 512 per vector step)
# with f32-accurate (x3) vs bf16 acting, two seeds each, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
O=gpurun_out/r03y; mkdir -p $O
for s in 0 1 2; do
  for act in x3 bf16; do
    timeout -k 10 240 python -u -m mazerl.train --envs 8192 --dim 81 --algo mixed --variant ddqn --steps 600 --batch 512 --updates-per-step 4 --log-every 0 --seed $s --acting $act | tail -1 | sed "s/^{/{\"acting\": \"$act\", \"seed\": $s, /" >> $O/cfg4_ab.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$O/cfg4_ab.jsonl'):
    d=json.loads(l); print(d['acting'], d['seed'], round(d['train_env_steps_per_s']/1e6,2), d['train_wins'], d['win_rate_greedy'], d['win_rate_greedy_best_of_6'])"
