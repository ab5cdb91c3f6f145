#!/bin/bash
# k_gram_chol_lag with rectangle tile ownership (NT = 15): mirror / lag / parity / BH tests, then the
# main line under rocprofv3 kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05aa}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_lag.py tests/test_gpu_parity.py tests/test_gpu_bh.py \
  -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_main_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst \
  > gpurun_out/prof_main_$TAG.json 2> gpurun_out/prof_main_$TAG.err
