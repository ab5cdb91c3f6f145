#!/bin/bash
# Ns = 5 tests, interleaved tile inverse (mirror bit-exactness + main-line time), full configs[3] OOS run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ns5.py tests/test_gpu_mirror.py tests/test_gpu_lag.py -v --timeout 300 \
  --timeout-method thread -s -rf > gpurun_out/r03_check13_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 10 > gpurun_out/r03_probe_main13.log 2>&1 || exit 1
OPENBLAS_NUM_THREADS=1 timeout -k 10 400 python -u tools/run_oos_full.py --no-maxlambda --out gpurun_out/r03h_oos_full.json \
  > gpurun_out/r03h_oos_full.log 2>&1
