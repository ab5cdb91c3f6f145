#!/bin/bash
# MFMA block products in k_sv_big's Cholesky + inverse: large-N parity tests, S120 sweep, then the timing probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bign.py tests/test_gpu_s120.py -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/r03_check_sv2.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/sv_probe2.log 2>&1
