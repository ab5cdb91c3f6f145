#!/bin/bash
# k_cta_solve_lag on two workgroups per chain at small B: lag / mirror / schedule bit-identity tests,
# then the floor phases (split default) and the one-workgroup floor for comparison.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05m}
timeout -k 10 900 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_lag.py tests/test_gpu_mirror.py \
  tests/test_gpu_bh.py -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
CCMM_SOLVE_SPLIT=0 timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_${TAG}_nosplit.json 2>> gpurun_out/floor_$TAG.err
