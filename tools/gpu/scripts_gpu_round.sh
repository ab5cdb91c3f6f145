#!/bin/bash
# round measurement: rocprofv3 kernel stats over the bench (all lines, no CPU baseline), then
# the default bench (the driver's command).  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02b}
rm -rf gpurun_out/prof_$TAG
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$R/bench.py" --no-cpu > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 5
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 4
