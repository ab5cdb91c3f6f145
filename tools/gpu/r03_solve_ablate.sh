#!/bin/bash
# k_cta_solve_big phase ablation at the S120 shape (B = 64): skip bits 1 v/U, 2 X'v, 4 forward,
# 8 backward, 16 residual (draws meaningless; timings only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sk in 0 1 2 4 8 16 31; do
  CCMM_SOLVE_SKIP=$sk timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/solve_ablate_$sk.log 2>&1 || exit $?
done
