#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_elb_wavefront.py tests/test_gpu_bh.py tests/test_gpu_gibbs_shadowrates.py \
  tests/test_gpu_gibbs_b3.py tests/test_gpu_gibbs_dense_psi.py tests/test_gpu_ps.py tests/test_gpu_ns5.py tests/test_gpu_hybrid.py \
  tests/test_gpu_shadowrate.py tests/test_gpu_vintages.py -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/r06f_tests.log 2>&1 || exit 1
for cfg in "elb_parts=1" "elb_parts=2"; do
  echo "== $cfg" >> gpurun_out/r06f_floor.log
  timeout -k 10 200 python -u tools/probe_floor.py 20 $cfg >> gpurun_out/r06f_floor.log 2>&1 || exit 1
done
