#!/bin/bash
# k_chol_big phase ablation at the S120 shape (B = 64): skip bits 1 update, 2 factor, 4 panel,
# 8 tile factor + inverse, 16 inverse off-diagonal tiles, 32 trailing tile updates (timings only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sk in 0 1 2 4 8 16 32; do
  CCMM_CHOL_SKIP=$sk timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/chol_ablate_$sk.log 2>&1 || exit $?
done
