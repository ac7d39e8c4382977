# round 3 final: k_step PMC passes for the current sources (profiles/collect.sh), then the HEAD
# check (profiles/r03_head2.sh: every GPU test, smoke, bench line, rocprofv3 stats, training
# trace, 2-rank rehearsal). Run under gpurun from the repo root.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh
RUN_TAG=${RUN_TAG:-r03zz4} bash profiles/r03_head2.sh
