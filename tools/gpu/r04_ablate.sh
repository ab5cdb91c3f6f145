#!/bin/bash
# Phase ablations (timing only; results invalid) of k_sv_part (CCMM_SV_MODE bits) and k_gram_chol_lag
# (CCMM_LAG_MODE 1 no SYRK, 2 no Cholesky) on the main line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04q}
OUT=gpurun_out/ablate_$TAG; mkdir -p $OUT
timeout -k 10 120 python tools/probe_main.py 256 3 > $OUT/base.log 2>&1 || exit $?
for m in 1 2 4 8 16 64; do
  CCMM_SV_MODE=$m timeout -k 10 120 python tools/probe_main.py 256 3 > $OUT/sv_$m.log 2>&1 || exit $?
done
for m in 1 2; do
  CCMM_LAG_MODE=$m timeout -k 10 120 python tools/probe_main.py 256 3 > $OUT/lag_$m.log 2>&1 || exit $?
done
