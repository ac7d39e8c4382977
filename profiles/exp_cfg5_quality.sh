# Round 4 (VERDICT next 7): config 5 quality — PPO on 4,096 toroidal 17..79 mazes, 3 seeds x 3,000
# vector steps, greedy win-rate on 1,000 fresh mazes and on 1,000 best-of-6 mazes.
set -o pipefail
export PYTHONPATH=$PWD/maze-solving-agent-gymnasium_amd:$PYTHONPATH
mkdir -p gpurun_out/r04e
for seed in 0 1 2; do
  timeout -k 10 400 python -u -m mazerl.train_ppo --envs 4096 --steps 3000 --eval-mazes 1000 --seed $seed \
    >> gpurun_out/r04e/cfg5_quality.jsonl 2>> gpurun_out/r04e/cfg5_quality.err || exit 1
done
