#!/bin/bash
# round-3 check 8: missingrate store (PS proposal 1), packed SV factors by default, QR-fallback sync cost
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_hybrid.py tests/test_gpu_parity.py \
  tests/test_gpu_shadowrate.py tests/test_gpu_fcst_hybrid.py -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/r03_check8_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 10 > gpurun_out/r03_probe_main8.log 2>&1 || exit 1
echo "no QR fallback sync" >> gpurun_out/r03_probe_main8.log
CCMM_NO_QR_FALLBACK=1 timeout -k 10 120 python -u tools/probe_main.py 256 10 >> gpurun_out/r03_probe_main8.log 2>&1
