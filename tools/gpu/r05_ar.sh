#!/bin/bash
# k_cta_solve_big phase ablation on the hybrid line (256 chains; timing only, ablation build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
out=gpurun_out/r05ar_solve_ablation.txt; : > $out
for s in 0 1 2 4 8 16; do
  echo "== CCMM_SOLVE_SKIP=$s" >> $out
  CCMM_SOLVE_SKIP=$s timeout -k 10 120 python tools/probe_hybrid.py 256 3 >> $out 2>&1 || exit 1
done
