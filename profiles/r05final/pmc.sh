#!/bin/bash
# round 5 final: k_step kernel traces + FETCH_SIZE / WRITE_SIZE passes at the final sources
# (profiles/collect.sh; summarised here by profiles/summarize.py into profiles/pmc_k_step.json)
set -o pipefail
bash profiles/collect.sh && ls gpurun_out/prof
