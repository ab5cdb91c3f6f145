#!/bin/bash
# A-step forms (real / N = 24 / T = 1100), A-step oracle parity incl. T = 1100, shadow-rate model real-data CRN
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ae}
timeout -k 10 600 python -u -m pytest tests/test_gpu_astep_forms.py "tests/test_gpu_parity.py::test_astep" \
  tests/test_gpu_shadowrate.py -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1
