#!/bin/bash
# k_chol_big update chunk width 4 (libccmm_ck4.so) against 8 (committed), hybrid line 256 chains
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/probe_hybrid.py 256 3 > gpurun_out/r05ba_ck8.txt 2>&1 &&
CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ck4.so timeout -k 10 120 python tools/probe_hybrid.py 256 3 \
  > gpurun_out/r05ba_ck4.txt 2>&1 &&
timeout -k 10 120 python tools/probe_hybrid.py 256 3 > gpurun_out/r05ba_ck8b.txt 2>&1
