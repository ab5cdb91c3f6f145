#!/bin/bash
# k_sv_part even LDS strides + ds_read_b128 pairs: SV tests, then main-line kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05au}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_sv_split.py tests/test_gpu_parity.py tests/test_gpu_mirror.py tests/test_gpu_bh.py \
  > gpurun_out/${TAG}_tests.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 10 > gpurun_out/${TAG}_main.txt 2>&1 &&
timeout -k 10 120 python tools/dbg/probe_linear.py 1 20 > gpurun_out/${TAG}_b1.txt 2>&1
