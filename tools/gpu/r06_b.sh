#!/bin/bash
# round 6: device-count probe, the multi-CU ELB parity tests, then the floor probe per ELB layout
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dbg/devcount_probe.py > gpurun_out/r06b_devcount.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_elb_wavefront.py -x -v --timeout 200 --timeout-method thread -s \
  > gpurun_out/r06b_elb_tests.log 2>&1 &&
for cfg in "elb_parts=1" "elb_parts=2" "elb_parts=4" "elb_parts=2 qr_fallback=0"; do
  echo "== $cfg" >> gpurun_out/r06b_floor.log
  timeout -k 10 200 python -u tools/probe_floor.py 20 $cfg >> gpurun_out/r06b_floor.log 2>&1 || exit 1
done
