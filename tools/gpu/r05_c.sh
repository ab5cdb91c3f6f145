#!/bin/bash
# ELB fast path (precomputed AS241 of the pass's uniforms) + k_ps_prop early exit: ELB / PS / truncnorm
# parity and schedule bit-identity, then the floor phases and the CTA-solve phase ablations at B = 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05c}
ABL=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_elb_wavefront.py tests/test_gpu_bh.py tests/test_gpu_ps.py \
  tests/test_gpu_parity.py tests/test_gpu_gibbs_shadowrates.py tests/test_gpu_gibbs_b3.py tests/test_gpu_ns5.py \
  -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
for m in "ELB_MODE=1" "LAG_MODE=16" "LAG_MODE=32" "LAG_MODE=64" "LAG_MODE=128"; do
  env CCMM_LIB=$ABL CCMM_$m timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_${TAG}_$m.json \
    2> gpurun_out/floor_${TAG}_$m.err || exit $?
done
