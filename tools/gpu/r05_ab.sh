#!/bin/bash
# k_gram_chol_lag SYRK / factor split (CCMM_LAG_MODE 2: SYRK only, 1: factor only; timing only) for
# the rectangle tile ownership (libccmm_ablation.so) and the round-robin one (libccmm_ablation_rr.so)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
L=$PWD/ccmmshadowratevar-code_amd/csrc
for lib in libccmm_ablation.so libccmm_ablation_rr.so; do
  for m in 0 2 1; do
    CCMM_LIB=$L/$lib CCMM_LAG_MODE=$m timeout -k 10 150 python tools/dbg/probe_linear.py 256 5 \
      > gpurun_out/r05ab_${lib}_$m.json
  done
done
