#!/bin/bash
# Lattice mvncdf for 4+ censored series: predictive-density GPU tests; then the LPT cost calibration.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04r}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py tests/test_gpu_fcst_hybrid.py -x -v \
  --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 400 python tools/calibrate_lpt.py gpurun_out/lpt_calibration_$TAG.json 12 4 > gpurun_out/lpt_$TAG.log 2>&1
