#!/bin/bash
# ub histogram of the floor's Gibbs draws (ablation build), then the whole GPU suite and smoke()
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06final}
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so CCMM_ELB_MODE=4096 timeout -k 10 200 python -u tools/dbg/elb_ubhist.py 5 > gpurun_out/ubhist_$TAG.json 2> gpurun_out/ubhist_$TAG.err &&
bash tools/gpu/r06_final_tests.sh
