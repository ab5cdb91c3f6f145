#!/bin/bash
# full GPU suite after the A-step Gram tiles (and this round's ELB / solve / SV changes), then the floor phases
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05r}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err
