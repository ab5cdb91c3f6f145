#!/bin/bash
# PHI block on the auxiliary stream + software-pipelined PS normals: block-hybrid / PS parity, the
# overlap bit-identity test, then the floor phases.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_bh.py tests/test_gpu_ps.py \
  tests/test_gpu_fcst_chain.py -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
CCMM_PHI_OVERLAP=0 timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_${TAG}_noov.json 2> gpurun_out/floor_${TAG}_noov.err
