#!/bin/bash
# timing-only phase ablations under rocprofv3: scripts_gpu_abl.sh <ENVVAR> <values...>
# PROBE (env): the python probe command (default: the S120 CTA probe, 8 chains)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
PROBE=${PROBE:-"tools/probe_s120_cta.py 8 2"}
V=$1; shift
for sk in "$@"; do
  rm -rf gpurun_out/prof_abl
  env $V=$sk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_abl" -o run --output-format csv -- python $PROBE > gpurun_out/abl_${V}_$sk.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_abl -name "*kernel_stats.csv" | head -1)
  cp $f gpurun_out/abl_${V}_$sk.csv
done
