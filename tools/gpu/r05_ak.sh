#!/bin/bash
# k_elb_cond with the lags' W / Q passes batched: ELB / BH / B3 / Ns=5 / S120 tests, BH256 kernel times, floor
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ak}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bh.py tests/test_gpu_gibbs_b3.py tests/test_gpu_gibbs_shadowrates.py \
  tests/test_gpu_ns5.py tests/test_gpu_elb_wavefront.py tests/test_gpu_s120.py tests/test_gpu_hybrid.py \
  -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 150 python tools/kernel_times_bh.py 256 1 3 > gpurun_out/bh256_$TAG.json 2> gpurun_out/bh256_$TAG.err &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
