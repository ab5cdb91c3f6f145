#!/bin/bash
# k_cta_solve_lag register-pressure rework: bit-exact mirror tests, then the main line with 8 and 16
# waves and the 8-wave form's phase ablations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04n}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_parity.py tests/test_gpu_bh.py tests/test_gpu_ps.py tests/test_gpu_gibbs_shadowrates.py tests/test_gpu_hybrid.py -x -v \
  --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/solve8_$TAG.log 2>&1 &&
CCMM_SOLVE_ASYNC=0 timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/solve8s_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/kernel_times_bh.py 256 1 3 > gpurun_out/bh256_$TAG.log 2>&1 &&
for m in 16 32 64 128; do
  CCMM_LAG_MODE=$m timeout -k 10 120 python tools/probe_main.py 256 3 > gpurun_out/solve_mode${m}_$TAG.log 2>&1 || exit $?
done
