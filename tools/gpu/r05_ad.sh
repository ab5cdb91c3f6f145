#!/bin/bash
# SYRK month order in 32-blocks (bank-conflict-free fragment reads): main-line kernel times
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 150 python tools/dbg/probe_linear.py 256 5 > gpurun_out/r05ad_linear.json
