#!/bin/bash
# round 5 (final k_step sources): k_step kernel traces + FETCH_SIZE / WRITE_SIZE passes per leg
# (profiles/collect.sh -> gpurun_out/prof; summarised by profiles/summarize.py into
# profiles/pmc_k_step.json)
set -o pipefail
timeout -k 10 1100 bash profiles/collect.sh && ls gpurun_out/prof
