#!/bin/bash
# timing experiment: the ELB draw's erfc replaced by a few-operation stand-in (results invalid)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_cheaperfc.so timeout -k 10 120 python tools/probe_floor.py 10 \
  > gpurun_out/floor_r05ai_cheaperfc.json
