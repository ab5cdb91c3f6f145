#!/bin/bash
# k_cta_solve_lag phase ablations (CCMM_LAG_MODE bits: 16 v_t, 32 X'v, 64 substitutions, 128 residual update)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 16 32 64 128 240; do
  echo "mode $m" >> gpurun_out/r03_ablate_solve.log
  CCMM_LAG_MODE=$m timeout -k 10 120 python -u tools/probe_main.py 256 5 >> gpurun_out/r03_ablate_solve.log 2>&1 || exit 1
done
