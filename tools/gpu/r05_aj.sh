#!/bin/bash
# solve back substitution with DPP lane exchanges: mirror / lag / schedule tests, main-line and floor timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05aj}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_lag.py tests/test_gpu_streams.py tests/test_gpu_bh.py \
  -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 150 python tools/dbg/probe_linear.py 256 5 > gpurun_out/linear_$TAG.json &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
