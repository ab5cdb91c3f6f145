#!/bin/bash
# S120 working points repeated (run-to-run spread of the s120 leg), bench.py's s120 leg only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04z}
for cfg in "112 4" "112 2" "96 2" "112 4" "112 2" "96 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --s120-only \
    --steps 2 --warmup 1 --s120-steps 3 --s120-chains $1 --s120-groups $2 >> gpurun_out/s120rep_$TAG.json 2>> gpurun_out/s120rep_$TAG.err || exit $?
done
