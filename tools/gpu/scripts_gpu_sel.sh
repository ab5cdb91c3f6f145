#!/bin/bash
# selected GPU tests (args: pytest selectors), one pytest process, own time limit
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/tests_sel.log 2>&1
rc=$?; echo "tests exit=$rc" >> gpurun_out/tests_sel.log; exit $rc
