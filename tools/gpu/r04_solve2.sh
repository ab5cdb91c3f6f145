#!/bin/bash
# k_cta_solve_lag weight prefetch: mirror / parity tests, main-line timing and phase ablations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04o}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_parity.py tests/test_gpu_bh.py -x -v \
  --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/solve8_$TAG.log 2>&1 &&
for m in 16 32 64 128; do
  CCMM_LAG_MODE=$m timeout -k 10 120 python tools/probe_main.py 256 3 > gpurun_out/solve_mode${m}_$TAG.log 2>&1 || exit $?
done
