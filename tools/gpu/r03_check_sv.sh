#!/bin/bash
# MFMA M_t / M_t'M_t in k_sv_big: large-N parity tests, S120 sweep, shadow-rate batch; then the S120 timing probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bign.py tests/test_gpu_s120.py tests/test_gpu_shadowrate_batch.py \
  tests/test_gpu_batch_native.py tests/test_gpu_post.py -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check_sv.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/sv_probe.log 2>&1
