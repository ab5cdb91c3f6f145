#!/bin/bash
# k_elb_cond with two waves for N <= 64: ELB / PS / batch parity, then BH kernel times (B = 256)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bh.py tests/test_gpu_elb_wavefront.py tests/test_gpu_ps.py \
  tests/test_gpu_gibbs_shadowrates.py tests/test_gpu_shadowrate.py tests/test_gpu_hybrid.py -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/r03_check_cond.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/kernel_times_bh.py 256 1 5 > gpurun_out/kt_bh256.json 2>&1
