#!/bin/bash
# round-3 check 4: full GPU suite (PS linear-term fix, unit-block substitutions, tiled k_chol_big
# diagonal, coalesced SV factor stores), main-line / SV-pack / hybrid / BH kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/r03_check4_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 5 > gpurun_out/r03_probe_main4.log 2>&1 || exit 1
CCMM_SV_MODE=128 timeout -k 10 120 python -u tools/probe_main.py 256 5 >> gpurun_out/r03_probe_main4.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/probe_hybrid.py 256 3 > gpurun_out/r03_probe_hybrid4.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/kernel_times_bh.py 256 1 3 > gpurun_out/r03_probe_bh4.log 2>&1
