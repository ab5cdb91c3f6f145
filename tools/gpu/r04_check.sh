#!/bin/bash
# round-4 check: large-N A-step on MFMA (bign / S120 parity), octet ELB kernel (identity + timing), S120 probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_bign.py tests/test_gpu_s120.py -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/bign_tests_$TAG.log 2>&1 || exit $?
TAG=$TAG bash tools/gpu/elb_lanes_probe.sh || exit $?
timeout -k 10 200 python tools/probe_s120_sweep.py 48 2 > gpurun_out/s120_probe_$TAG.txt 2>&1
