#!/bin/bash
# ELB wavefront cycle attribution at the floor (ablation build): full draws, then no draws
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 64 65; do
  CCMM_ELB_MODE=$m timeout -k 10 240 python tools/dbg/elb_prof.py 5 >> gpurun_out/r05h_elb_prof.txt
done
