#!/bin/bash
# End-of-round measurement: PMC summary (pmc_main.sh), the default bench.py run (the driver's command),
# and the main line under rocprofv3 --kernel-trace --stats.  Each GPU step under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04t}
TAG=$TAG bash tools/gpu/pmc_main.sh &&
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
rm -rf gpurun_out/prof_main_$TAG &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_main_$TAG" -o run --output-format csv -- python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst > gpurun_out/prof_main_$TAG.json 2> gpurun_out/prof_main_$TAG.err
