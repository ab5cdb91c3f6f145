#!/bin/bash
# k_sv_part phase ablation on the main line (256 chains; timing only, ablation build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
out=gpurun_out/r05at_sv_ablation.txt; : > $out
for s in 0 1 2 4 8 16 32; do
  echo "== CCMM_SV_MODE=$s" >> $out
  CCMM_SV_MODE=$s timeout -k 10 120 python tools/probe_main.py 256 5 >> $out 2>&1 || exit 1
done
