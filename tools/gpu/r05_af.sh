#!/bin/bash
# PS proposals with paired Box-Muller normals: PS / batch / OOS tests, floor phases
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ah}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_batch_native.py tests/test_gpu_oos.py \
  tests/test_gpu_shadowrate_batch.py tests/test_gpu_mcse_bh.py -x -v --timeout 300 --timeout-method thread -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
