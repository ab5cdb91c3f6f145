#!/bin/bash
# the whole GPU suite and smoke() on the final tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06final}
timeout -k 10 1000 python -u -m pytest -v -m gpu --timeout 240 --timeout-method thread tests/ > gpurun_out/full_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/full_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
