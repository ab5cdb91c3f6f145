#!/bin/bash
# A-step wave-parallel kernel: parity tests, A/B timing against k_astep (CCMM_ASTEP_V1=1) on the main
# line, then the instruction-issue counters of the block-hybrid sweep (pmc_issue.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04l}
timeout -k 10 500 python -u -m pytest tests/test_gpu_astep_forms.py tests/test_gpu_parity.py tests/test_gpu_mirror.py tests/test_gpu_bign.py \
  tests/test_gpu_distributed_nccl.py -x -v --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
CCMM_ASTEP_V1=1 timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/astep_v1_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/astep_w_$TAG.log 2>&1 &&
TAG=$TAG bash tools/gpu/pmc_issue.sh
