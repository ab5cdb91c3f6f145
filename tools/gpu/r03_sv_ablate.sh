#!/bin/bash
# k_sv_big phase ablation at the S120 shape (B = 64): skip bits 1 GEMM, 2 Gram, 4 chol+inverse,
# 8 w_t, 16 backward pass, 32 Linv store (draws meaningless; timings only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sk in 0 1 2 4 40 16 63; do
  CCMM_SV_SKIP=$sk timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/sv_ablate_$sk.log 2>&1 || exit $?
done
