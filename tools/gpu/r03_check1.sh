#!/bin/bash
# round-3 check: new drop-ins / tests, then the full configs[3] OOS run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aswitching.py tests/test_gpu_girf.py tests/test_gpu_fcst_hybrid.py \
  tests/test_gpu_mcse_real.py tests/test_gpu_fcst_chain.py tests/test_gpu_hybrid.py \
  -k "not bh]" -v --timeout 300 --timeout-method thread -s > gpurun_out/r03_check1_tests.log 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
OPENBLAS_NUM_THREADS=1 timeout -k 10 900 python -u tools/run_oos_full.py --out gpurun_out/r03_oos_full.json > gpurun_out/r03_oos_full.log 2>&1
