set -o pipefail
bash profiles/collect.sh && bash profiles/train_trace.sh && bash profiles/cfg2_trace2.sh gpurun_out/r04j
