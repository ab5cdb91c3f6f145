#!/bin/bash
# Ablation sweep of the lag CTA kernels (timing only; ablated runs give invalid draws).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for m in ${MODES:-0 1 2 4 6 16 32 64 128}; do
  echo "mode=$m" >> gpurun_out/ablate.log
  CCMM_LAG_MODE=$m timeout -k 10 120 python tools/kernel_times.py 256 2 6 >> gpurun_out/ablate.log 2>&1 || exit 2
done
