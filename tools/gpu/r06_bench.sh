#!/bin/bash
# default bench.py run (the driver's command) on the current tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06a}
timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
