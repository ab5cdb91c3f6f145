#!/bin/bash
# round-3 check 6: deterministic Newton pivot (bit-exact factor, 1e-9 sweep), native batch loop,
# main-line kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_batch_native.py \
  -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check6_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 5 > gpurun_out/r03_probe_main6.log 2>&1
