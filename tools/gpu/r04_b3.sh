#!/bin/bash
# gibbsdrawShadowratesB3 and the lattice mvncdf: their GPU tests, plus the ELB tests of the shared kernels;
# then the LPT cost calibration.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04s}
timeout -k 10 500 python -u -m pytest tests/test_gpu_gibbs_b3.py tests/test_gpu_fcst.py tests/test_gpu_gibbs_shadowrates.py \
  tests/test_gpu_elb_wavefront.py tests/test_gpu_bh.py tests/test_gpu_ps.py -x -v --timeout 200 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 400 python tools/calibrate_lpt.py gpurun_out/lpt_calibration_$TAG.json 12 4 > gpurun_out/lpt_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/kernel_times_bh.py 256 1 3 > gpurun_out/bh256_async_$TAG.log 2>&1 &&
CCMM_ELB_ASYNC=0 timeout -k 10 120 python tools/kernel_times_bh.py 256 1 3 > gpurun_out/bh256_lock_$TAG.log 2>&1
