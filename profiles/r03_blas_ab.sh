# round 3: config 5 and the DDQN training leg with torch's f32 GEMMs on rocBLAS vs hipBLASLt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT/maze-solving-agent-gymnasium_amd:$PYTHONPATH"
O=gpurun_out/r03bl; mkdir -p $O
for r in 1 2; do
  for lt in 1 0; do
    TORCH_BLAS_PREFER_HIPBLASLT=$lt timeout -k 10 300 python -u -m mazerl.train_ppo --envs 4096 --steps 600 > $O/cfg5_lt${lt}_$r.jsonl 2> $O/cfg5_lt${lt}_$r.err || { tail -20 $O/cfg5_lt${lt}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_lt${lt}_$r.jsonl').read().strip().splitlines()[-1]); print('cfg5 hipblaslt=$lt', round(d['train_env_steps_per_s']/1e6,3))"
  done
done
B="--legs bits --steps 20 --warmup 5 --no-cpu-baseline --eval-mazes 200"
for lt in 1 0; do
  TORCH_BLAS_PREFER_HIPBLASLT=$lt timeout -k 10 240 python -u bench.py $B > $O/ddqn_lt$lt.json 2> $O/ddqn_lt$lt.err || { tail -20 $O/ddqn_lt$lt.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ddqn_lt$lt.json'))['win_rate']; print('ddqn hipblaslt=$lt', round(d['train_env_steps_per_s']/1e6,2), d['greedy'])"
done
# the headline step past the 256 MB Infinity Cache: 131,072 instances (354 MB of f32 windows per step)
timeout -k 10 300 python -u bench.py --envs 131072 --legs window,bits --train-steps 0 --no-cpu-baseline > $O/bench_131072.json 2> $O/bench_131072.err || { tail -20 $O/bench_131072.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_131072.json')); print('131072', d['value'], d['ms_per_step'], d['roofline']['frac'], d['bits_mode']['value'], d['bits_mode']['roofline']['frac'])"
