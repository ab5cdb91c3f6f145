#!/bin/bash
# S120 per-kernel times without stream-group contention; full configs[3] OOS run (1 GPU)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe_s120_sweep.py 64 2 > gpurun_out/r03_probe_s120.log 2>&1 || exit 1
OPENBLAS_NUM_THREADS=16 timeout -k 10 600 python -u tools/run_oos_full.py --out gpurun_out/r03h_oos_full.json \
  > gpurun_out/r03h_oos_full.log 2>&1
