#!/bin/bash
# ELB wavefront cycle attribution under timing-only ablations (128 no record loads, 256 no predecessor
# wait, 512 no month sums, 1 no draws)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 64 192 320 576 960 65 193 449; do
  CCMM_ELB_MODE=$m timeout -k 10 240 python tools/dbg/elb_prof.py 5 >> gpurun_out/r05j_elb_prof.txt
done
