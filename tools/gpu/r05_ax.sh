#!/bin/bash
# k_sv_part NN = 20 phase-A block products on MFMA: SV / sweep tests, then main-line and B = 1 kernel
# times with and without (CCMM_SV_MFMA=0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ax}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_sv_split.py tests/test_gpu_parity.py tests/test_gpu_mirror.py tests/test_gpu_bh.py \
  tests/test_gpu_shadowrate.py tests/test_gpu_mcse.py > gpurun_out/${TAG}_tests.log 2>&1 &&
timeout -k 10 120 python tools/probe_main.py 256 10 > gpurun_out/${TAG}_main.txt 2>&1 &&
CCMM_SV_MFMA=0 timeout -k 10 120 python tools/probe_main.py 256 10 > gpurun_out/${TAG}_main_valu.txt 2>&1 &&
timeout -k 10 120 python tools/dbg/probe_linear.py 1 20 > gpurun_out/${TAG}_b1.txt 2>&1 &&
CCMM_SV_MFMA=0 timeout -k 10 120 python tools/dbg/probe_linear.py 1 20 > gpurun_out/${TAG}_b1_valu.txt 2>&1
