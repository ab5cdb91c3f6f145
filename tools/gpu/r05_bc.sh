#!/bin/bash
# mirror / shadow-rate real-data checks on the rebuilt library, then the end-of-round measurement
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05bc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_shadowrate.py -x -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
TAG=$TAG bash tools/gpu/final_bench.sh
