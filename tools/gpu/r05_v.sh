#!/bin/bash
# X'v with sixteen months per LDS round trip: lag / mirror / schedule tests, floor phases, attribution
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05y}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lag.py tests/test_gpu_mirror.py tests/test_gpu_streams.py \
  -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
timeout -k 10 60 ./tools/dbg/latency_calib > gpurun_out/latency_calib.json &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so timeout -k 10 120 python tools/dbg/floor_phase_prof.py 5 \
  > gpurun_out/phase_prof_$TAG.json
