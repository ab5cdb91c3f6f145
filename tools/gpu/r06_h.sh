#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py \
  tests/test_gpu_batch_native.py tests/test_gpu_oos.py -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/r06h_tests.log 2>&1 || exit 1
for cfg in "elb_spec=0 fcst_overlap=0" "elb_spec=0" "elb_spec=1" "elb_spec=0 noprof" "elb_spec=1 noprof"; do
  echo "== $cfg" >> gpurun_out/r06h_floor.log
  timeout -k 10 200 python -u tools/probe_floor.py 20 $cfg >> gpurun_out/r06h_floor.log 2>&1 || exit 1
done
