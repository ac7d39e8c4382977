set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 300 python -u profiles/exp_mcclendon.py > $O/mcc_timing.json 2> $O/mcc_timing.err || { tail -20 $O/mcc_timing.err; exit 1; }
cat $O/mcc_timing.json
