#!/bin/bash
# ELB multi-CU kernel at the floor under timing-only ablations (ablation build): 0 none, 256 no
# predecessor wait, 1024 the month sums twice, 2048 every draw twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06f}
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 256 1024 2048; do
  echo "mode $m" >> gpurun_out/elbabl_$TAG.txt
  CCMM_ELB_MODE=$m timeout -k 10 200 python -u tools/probe_floor.py 6 >> gpurun_out/elbabl_$TAG.txt 2>> gpurun_out/elbabl_$TAG.err || exit 1
done
