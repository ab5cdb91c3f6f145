#!/bin/bash
# kernel stats of the main + predictive lines (k_fcst vs k_fcst_scores split at B = 256)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05al}
rm -rf gpurun_out/prof_pred_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pred_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 \
  > gpurun_out/prof_pred_$TAG.json 2> gpurun_out/prof_pred_$TAG.err
