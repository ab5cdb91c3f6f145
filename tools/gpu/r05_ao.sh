#!/bin/bash
# kernel stats of the hybrid line alone (256 chains): where the 26 ms sweep goes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05ao}
rm -rf gpurun_out/prof_hy_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_hy_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --steps 1 --warmup 0 --no-fcst --bh-steps 0 --hy-steps 3 --hy-chains 256 \
  --oos-steps 0 --oos-full-draws 0 --s120-steps 0 --girf-draws 0 \
  > gpurun_out/prof_hy_$TAG.json 2> gpurun_out/prof_hy_$TAG.err
