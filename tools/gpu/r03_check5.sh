#!/bin/bash
# round-3 check 5: device-order factor mirror (bit-exact factor record, 1e-9 sweep), native batch
# loop (ccmm_run_batch) vs the Python driver, lag-path parity, main-line kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_batch_native.py tests/test_gpu_lag.py \
  tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check5_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 5 > gpurun_out/r03_probe_main5.log 2>&1
