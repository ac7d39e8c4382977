# round 3: PMC / kernel-trace collection (both env-step legs) + config 5 PPO with the on-device
# rollout (f32 acting) — throughput, win-rate and a phase breakdown
set -o pipefail
export PYTHONPATH="$PWD/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
O=gpurun_out/r03b; mkdir -p $O
bash profiles/collect.sh && echo collect-ok
timeout -k 10 600 python -u -m mazerl.train_ppo --envs 4096 --steps 600 > $O/ppo_cfg5.jsonl 2> $O/ppo_cfg5.err || { tail -20 $O/ppo_cfg5.err; exit 1; }
tail -2 $O/ppo_cfg5.jsonl
timeout -k 10 600 python -u profiles/ppo_breakdown.py > $O/ppo_breakdown.json 2> $O/ppo_breakdown.err || { tail -20 $O/ppo_breakdown.err; exit 1; }
cat $O/ppo_breakdown.json
