#!/bin/bash
# k_sv_part with the X-solve rows read one row ahead: SV parity / bit-identity tests and main-line timing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_parity.py tests/test_gpu_bign.py -x -v \
  --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 5 > gpurun_out/main_$TAG.log 2>&1
