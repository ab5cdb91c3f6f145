#!/bin/bash
# round-3 check 2: mirror parity, hybrid predictive density, hybrid Cholesky ablations, full OOS run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_fcst_hybrid.py tests/test_gpu_parity.py \
  -v --timeout 300 --timeout-method thread -s > gpurun_out/r03_check2_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for m in 0 1 2 4; do
  CCMM_CHOL_SKIP=$m timeout -k 10 120 python -u tools/probe_hybrid.py 256 3 >> gpurun_out/r03_probe_hybrid.log 2>&1 || exit 1
done
CCMM_GC18=1 timeout -k 10 120 python -u tools/probe_hybrid.py 256 3 >> gpurun_out/r03_probe_hybrid.log 2>&1 || exit 1
CCMM_GC18=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -x -v --timeout 200 --timeout-method thread -s > gpurun_out/r03_gc18_tests.log 2>&1
OPENBLAS_NUM_THREADS=1 timeout -k 10 1000 python -u tools/run_oos_full.py --out gpurun_out/r03_oos_full.json > gpurun_out/r03_oos_full.log 2>&1
