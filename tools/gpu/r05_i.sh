#!/bin/bash
# ELB month sums as one interleaved DPP reduction (wave_sum_dpp_n): bit-identity / parity tests of the
# ELB kernels, the cycle attribution (ablation build) and the floor phases.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05l}
timeout -k 10 900 python -u -m pytest tests/test_gpu_elb_wavefront.py tests/test_gpu_gibbs_shadowrates.py \
  tests/test_gpu_mirror.py tests/test_gpu_ns5.py tests/test_gpu_bh.py tests/test_gpu_ps.py \
  -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so CCMM_ELB_MODE=64 timeout -k 10 240 \
  python tools/dbg/elb_prof.py 5 > gpurun_out/elb_prof_$TAG.json &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
