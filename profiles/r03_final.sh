# round 3 final: k_step PMC passes for the current sources (profiles/collect.sh), then the HEAD
# check (profiles/r03_head2.sh: every GPU test, smoke, bench line, rocprofv3 stats, training
# trace, 2-rank rehearsal). Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh
for leg in window bits; do
  python3 profiles/summarize.py ${RUN_TAG:-r03zz4}_$leg gpurun_out/prof/kt_$leg gpurun_out/prof/fetch_$leg gpurun_out/prof/write_$leg --envs 65536 --dim 81 --mode $leg > /dev/null
done
RUN_TAG=${RUN_TAG:-r03zz4} bash profiles/r03_head2.sh
