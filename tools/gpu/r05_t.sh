#!/bin/bash
# solve / A-step phase attribution at the floor (ablation build), split and one-workgroup solve
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
timeout -k 10 120 python tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_prof_r05t.json
CCMM_SOLVE_SPLIT=0 timeout -k 10 120 python tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_prof_r05t_nosplit.json
