#!/bin/bash
# k_elb_gibbs lane kernel vs wave kernel: bit-identity test, then per-kernel times at B = 256 / 1024.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_elb_wavefront.py -v --timeout 200 --timeout-method thread -s \
  > gpurun_out/elb_lanes_tests_$TAG.log 2>&1 || exit $?
for B in 256 512 1024; do
  for L in 0 2; do
    CCMM_ELB_OCT=$L timeout -k 10 120 python tools/kernel_times_bh.py $B 1 3 0 > gpurun_out/elb_lanes_B${B}_L${L}_$TAG.json 2>&1 || exit $?
  done
done
