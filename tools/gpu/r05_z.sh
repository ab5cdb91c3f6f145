#!/bin/bash
# main line (linear, 256 chains) under rocprofv3 kernel stats after this round's kernel changes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05z}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_main_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst \
  > gpurun_out/prof_main_$TAG.json 2> gpurun_out/prof_main_$TAG.err
