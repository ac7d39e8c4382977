# round 3: PPO fused head loss + per-location minibatch graphs — tests, then config 5 A/B
# (MZ_PPO_FUSED_LOSS=1 vs 0, interleaved) and the phase breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_agents.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for f in 1 0; do
    MZ_PPO_FUSED_LOSS=$f timeout -k 10 300 python -u -m mazerl.train_ppo --envs 4096 --steps 600 > $O/cfg5_f${f}_$r.jsonl 2> $O/cfg5_f${f}_$r.err || { tail -20 $O/cfg5_f${f}_$r.err; exit 1; }
    tail -1 $O/cfg5_f${f}_$r.jsonl | cut -c1-400
  done
done
timeout -k 10 300 python -u profiles/ppo_breakdown.py > $O/breakdown.json 2> $O/breakdown.err || { tail -20 $O/breakdown.err; exit 1; }
cat $O/breakdown.json
