#!/bin/bash
# solve / A-step phase attribution at the floor (ablation build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06d}
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
timeout -k 10 200 python -u tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.err
