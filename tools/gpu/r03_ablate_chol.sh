#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 2 8 16 32 56; do
  echo "skip $m" >> gpurun_out/r03_ablate_chol.log
  CCMM_CHOL_SKIP=$m timeout -k 10 120 python -u tools/probe_hybrid.py 256 2 >> gpurun_out/r03_ablate_chol.log 2>&1 || exit 1
done
