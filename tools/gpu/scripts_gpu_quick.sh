#!/bin/bash
# quick GPU iteration: selected GPU tests (args, default all) then per-kernel timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests exit=$rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/kernel_times.py 256 2 6 > gpurun_out/ktimes.log 2>&1
rc=$?; echo "ktimes exit=$rc" >> gpurun_out/ktimes.log; exit $rc
