#!/bin/bash
# k_elb_cond with four waves for N > 64, SV diag-block pivots without division: ELB / PS / large-N parity, S120 probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bign.py tests/test_gpu_s120.py tests/test_gpu_bh.py tests/test_gpu_elb_wavefront.py \
  tests/test_gpu_ps.py tests/test_gpu_ns5.py tests/test_gpu_gibbs_shadowrates.py -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/r03_check_elb.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/sv_probe3.log 2>&1
