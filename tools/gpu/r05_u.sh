#!/bin/bash
# solve phase attribution with the X'v loop skipped (CCMM_LAG_MODE=32, timing only)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
CCMM_LAG_MODE=32 timeout -k 10 120 python tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_prof_r05u_lag32.json
