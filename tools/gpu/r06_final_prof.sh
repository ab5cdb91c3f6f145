#!/bin/bash
# end-of-round counters and kernel statistics of the main line: the PMC passes (tools/gpu/pmc_main.sh,
# profiles/${TAG}_pmc.json) and one rocprofv3 --kernel-trace --stats run of the bench's main line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06zz}
TAG=$TAG bash tools/gpu/pmc_main.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_main_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --oos-full-draws 0 --s120-steps 0 --girf-draws 0 --no-fcst \
  > gpurun_out/prof_main_$TAG.json 2> gpurun_out/prof_main_$TAG.err
