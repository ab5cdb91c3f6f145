#!/bin/bash
# k_elb_prep rows over several workgroups at small B; k_ps_prop with the band factor in LDS and four
# accumulators: ELB / PS / block-hybrid parity and bit-identity tests, then the floor phases.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05g}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_bh.py tests/test_gpu_elb_wavefront.py \
  tests/test_gpu_streams.py tests/test_gpu_ns5.py tests/test_gpu_gibbs_shadowrates.py tests/test_gpu_oos.py \
  -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
