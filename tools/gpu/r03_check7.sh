#!/bin/bash
# round-3 check 7: batched rhs loads / table-free residual update in k_cta_solve_lag (mirror + lag parity, times)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_lag.py tests/test_gpu_parity.py \
  -v --timeout 200 --timeout-method thread -s -rf > gpurun_out/r03_check7_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for m in 0 32 128; do
  echo "mode $m" >> gpurun_out/r03_probe_main7.log
  CCMM_LAG_MODE=$m timeout -k 10 120 python -u tools/probe_main.py 256 5 >> gpurun_out/r03_probe_main7.log 2>&1 || exit 1
done
