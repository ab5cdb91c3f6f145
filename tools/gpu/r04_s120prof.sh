#!/bin/bash
# Per-kernel device times of S120 sweeps (48 chains, one stream group) under rocprofv3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04y}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s120_$TAG -o s120 -- python3 tools/probe_s120_sweep.py 48 2 \
  > gpurun_out/s120prof_$TAG.log 2>&1
