#!/bin/bash
# timing-only phase ablations under rocprofv3: scripts_gpu_abl.sh <ENVVAR> <values...>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=$1; shift
for sk in "$@"; do
  rm -rf gpurun_out/prof_abl
  env $V=$sk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_abl" -o run --output-format csv -- python tools/probe_s120_cta.py 8 2 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_abl -name "*kernel_stats.csv" | head -1)
  cp $f gpurun_out/abl_${V}_$sk.csv
done
