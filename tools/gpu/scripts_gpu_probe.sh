#!/bin/bash
# rocprofv3 kernel stats of a probe script: scripts_gpu_probe.sh <tag> <script> [args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
rm -rf gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$@" > gpurun_out/probe_$TAG.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/probe_$TAG.log
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/stats_$TAG.csv
exit $rc
