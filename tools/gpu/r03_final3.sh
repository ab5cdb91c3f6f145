#!/bin/bash
# end-of-round confirmation: full GPU suite and smoke() on the committed tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_r03k.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r03k.log 2>&1
