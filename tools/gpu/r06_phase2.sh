#!/bin/bash
# solve phase attribution under timing-only ablations of the lag solve (CCMM_LAG_MODE 32: no X'v, 16: no v_t)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06e}
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 32 16 48; do
  CCMM_LAG_MODE=$m timeout -k 10 200 python -u tools/dbg/floor_phase_prof.py 5 >> gpurun_out/phase_$TAG.json 2>> gpurun_out/phase_$TAG.err || exit 1
done
