#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mirror.py tests/test_gpu_bh.py -v --timeout 200 \
  --timeout-method thread -s -rf > gpurun_out/r03_check11_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 10 > gpurun_out/r03_probe_main11.log 2>&1
