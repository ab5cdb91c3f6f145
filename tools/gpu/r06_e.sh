#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_elb_wavefront.py -x -v --timeout 200 --timeout-method thread -s \
  > gpurun_out/r06e_tests.log 2>&1 || exit 1
for cfg in "elb_parts=1" "elb_parts=2" "elb_parts=4"; do
  echo "== $cfg" >> gpurun_out/r06e_floor.log
  timeout -k 10 200 python -u tools/probe_floor.py 20 $cfg >> gpurun_out/r06e_floor.log 2>&1 || exit 1
done
