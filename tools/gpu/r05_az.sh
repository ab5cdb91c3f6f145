#!/bin/bash
# S120 line with the k_chol_big panel prefetch (libccmm_panelpf.so) against the committed library
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --s120-only > gpurun_out/r05az_s120_base.json 2> gpurun_out/r05az_s120_base.err &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_panelpf.so timeout -k 10 300 python bench.py --s120-only \
  > gpurun_out/r05az_s120_pf.json 2> gpurun_out/r05az_s120_pf.err
