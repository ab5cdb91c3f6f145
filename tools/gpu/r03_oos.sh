#!/bin/bash
# full configs[3] OOS run on one GPU (host LAPACK max-root pool single-threaded BLAS per worker)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
OPENBLAS_NUM_THREADS=1 timeout -k 10 600 python -u tools/run_oos_full.py --out gpurun_out/r03h_oos_full.json \
  > gpurun_out/r03h_oos_full.log 2>&1
