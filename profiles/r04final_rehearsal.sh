# Round 4, final sources: the 4-rank rehearsal of the whole bench through its own launcher, all
# ranks on the one GPU over gloo (the 8-GPU RCCL runs are the driver's)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04final_rh; mkdir -p $out
MZ_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench.py --gpus 4 --envs 16384 --cfg4-envs 2048 --cfg5-envs 1024 --curriculum-envs 1024 --curriculum-steps 600 --eval-mazes 300 --cfg-eval-mazes 200 > $out/bench4.json 2> $out/bench4.err
