#!/bin/bash
# ELB wavefront with the month-record head in LDS and 16 passes in flight at small B: bit-identity tests,
# floor kernel times per wave count, block-hybrid line kernel times at B = 256.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04x}
timeout -k 10 500 python -u -m pytest tests/test_gpu_elb_wavefront.py tests/test_gpu_bh.py tests/test_gpu_gibbs_shadowrates.py \
  -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
for w in 8 16; do
  CCMM_ELB_WAVES=$w timeout -k 10 200 python tools/probe_floor.py 10 > gpurun_out/floor_w${w}_$TAG.json 2>&1 || exit $?
done &&
timeout -k 10 200 python tools/kernel_times_bh.py 256 > gpurun_out/bh256_$TAG.json 2>&1
