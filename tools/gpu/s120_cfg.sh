#!/bin/bash
# S120 line at several (chains, stream groups) working points (bench.py's s120 leg only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04u}
for cfg in "96 1" "96 3" "112 2" "112 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --s120-only \
    --steps 2 --warmup 1 --s120-chains $1 --s120-groups $2 > gpurun_out/s120_${1}_${2}_$TAG.json 2> gpurun_out/s120_${1}_${2}_$TAG.err || exit $?
done
