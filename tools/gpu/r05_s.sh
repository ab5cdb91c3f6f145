#!/bin/bash
# A-step Gram tiles with the weight prefetch ring: A-step / parity tests, then the floor phases
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_astep_forms.py tests/test_gpu_parity.py tests/test_gpu_bh.py \
  -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so timeout -k 10 120 python tools/dbg/floor_phase_prof.py 5 > gpurun_out/phase_prof_$TAG.json
