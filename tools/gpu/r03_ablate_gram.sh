#!/bin/bash
# k_gram_chol_lag phase ablations (CCMM_LAG_MODE bits: 1 no SYRK, 2 no Cholesky, 256 no 16x16 tile factor/inverse,
# 1024 no look-ahead/trailing updates); timing only
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 1 2 256 1024 1280; do
  echo "mode $m" >> gpurun_out/r03_ablate_gram.log
  CCMM_LAG_MODE=$m timeout -k 10 120 python -u tools/probe_main.py 256 5 >> gpurun_out/r03_ablate_gram.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_mcse_real.py tests/test_gpu_batch_native.py -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/r03_mcse_tests.log 2>&1
