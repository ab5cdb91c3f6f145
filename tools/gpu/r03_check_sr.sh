#!/bin/bash
# shadow-rate VAR vintage batch (ccmm_chains_summaries_floor), pooled linear MCSE fixture, summaries regression
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shadowrate_batch.py tests/test_gpu_shadowrate.py \
  tests/test_gpu_batch_native.py tests/test_gpu_post.py tests/test_gpu_mcse_real.py -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/r03_check_sr.log 2>&1
