#!/bin/bash
# Ns = 5 (PS band width 65), PS / forecast parity after the Genz clamp, full configs[3] OOS run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ns5.py tests/test_gpu_ps.py tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py \
  tests/test_gpu_fcst_hybrid.py -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check14_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
OPENBLAS_NUM_THREADS=1 timeout -k 10 400 python -u tools/run_oos_full.py --no-maxlambda --out gpurun_out/r03h_oos_full.json \
  > gpurun_out/r03h_oos_full.log 2>&1
