#!/bin/bash
# GPU test step: pytest over the given test selection (default: the whole -m gpu suite), its own time
# limit, log under gpurun_out/.  Usage: TAG=r04a bash tools/gpu/tests.sh [pytest args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
LIMIT=${LIMIT:-700}
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
timeout -k 10 "$LIMIT" python -u -m pytest "${ARGS[@]}" -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
