#!/bin/bash
# Ablation sweeps (timing only; ablated runs give invalid draws):
#   LMODES -> CCMM_LAG_MODE (lag CTA kernels), SMODES -> CCMM_SV_MODE (SV sampler phases)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; : > gpurun_out/ablate.log
for m in ${LMODES:-}; do
  echo "lag mode=$m" >> gpurun_out/ablate.log
  CCMM_LAG_MODE=$m timeout -k 10 120 python tools/kernel_times.py 256 2 6 >> gpurun_out/ablate.log 2>&1 || exit 2
done
for m in ${SMODES:-}; do
  echo "sv mode=$m" >> gpurun_out/ablate.log
  CCMM_SV_MODE=$m timeout -k 10 120 python tools/kernel_times.py 256 2 6 >> gpurun_out/ablate.log 2>&1 || exit 2
done
