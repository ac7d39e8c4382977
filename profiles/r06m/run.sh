#!/bin/bash
# round 6: curriculum legs that fire and learn — epsilon_decay scale, instances and length
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06m
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, then bench args
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs bits --no-cpu-baseline --train-steps 0 \
    --config-legs "" --eval-mazes 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 - $O/$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d.items():
    if not k.startswith("curriculum_leg"):
        continue
    print(json.dumps({"run": sys.argv[2], "leg": k, "envs": v["envs_per_gpu"], "steps": v["train_vector_steps"],
                      "decay": v["epsilon_decay"], "sps": round(v["train_env_steps_per_s"]),
                      "wins": v["total_wins"], "median": v.get("wins_per_instance_median"),
                      "at_end": v["instances_per_algorithm_at_end"], "greedy": v["greedy_by_algorithm"],
                      "infer": {a: v["infer_by_algorithm"][a]["greedy"] for a in ("r-prim", "prim&kill", "dfs")},
                      "seen": v["seen_mazes_reference_protocol"].get("greedy")}), flush=True)
PY
}
run ${1:-pi40_2048_40k} --curriculum-rules per-instance --curriculum-decay-div 40 --curriculum-pi-envs 2048 --curriculum-pi-steps 40000 --curriculum-pi-updates 2 && \
run pi40_1024_60k --curriculum-rules per-instance --curriculum-decay-div 40 --curriculum-pi-envs 1024 --curriculum-pi-steps 60000 --curriculum-pi-updates 2 && \
run gl40_12k --curriculum-rules global --curriculum-decay-div 40 --curriculum-steps 12000
