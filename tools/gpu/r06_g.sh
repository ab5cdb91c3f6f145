#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_elb_wavefront.py tests/test_gpu_ps.py \
  tests/test_gpu_mcse_bh.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r06g_tests.log 2>&1 || exit 1
for cfg in "elb_spec=0" "elb_spec=1"; do
  echo "== $cfg" >> gpurun_out/r06g_floor.log
  timeout -k 10 200 python -u tools/probe_floor.py 20 $cfg >> gpurun_out/r06g_floor.log 2>&1 || exit 1
done
