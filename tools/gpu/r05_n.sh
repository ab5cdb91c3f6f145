#!/bin/bash
# k_sv_part phase attribution at the floor (ablation build, timing only): phase A off (1), separator
# pass off (2), separator back-substitution off (4), segment back-substitution off (8), g recursion off (16)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 1 2 4 8 16 6; do
  CCMM_SV_MODE=$m timeout -k 10 120 python tools/probe_floor.py 5 > gpurun_out/r05n_sv_mode_$m.json
done
