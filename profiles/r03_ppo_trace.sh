# round 3: rocprofv3 kernel trace of the config-5 PPO trainer (4,096 toroidal 17..79, 300 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 -m mazerl.train_ppo --envs 4096 --steps 300 --eval-mazes 64 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
tail -2 $O/kt.log
