#!/bin/bash
# End-of-round confirmation: full GPU suite, smoke(), main-line rocprofv3 kernel stats.  Each GPU step
# has its own time limit; the steps are chained so the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 &&
rm -rf gpurun_out/prof_main_$TAG &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_main_$TAG" -o run --output-format csv -- python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 --no-fcst > gpurun_out/prof_main_$TAG.json 2> gpurun_out/prof_main_$TAG.err
