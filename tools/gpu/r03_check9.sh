#!/bin/bash
# round-3 check 9: k_chol_big tile factor with fast pivots / register inverse (hybrid K = 277, S120 K = 1441)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_hybrid.py tests/test_gpu_bign.py \
  tests/test_gpu_s120.py -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check9_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for m in 0 1 2 4; do
  CCMM_CHOL_SKIP=$m timeout -k 10 120 python -u tools/probe_hybrid.py 256 3 >> gpurun_out/r03_probe_hybrid9.log 2>&1 || exit 1
done
