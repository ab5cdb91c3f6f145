#!/bin/bash
# round 6: parity of the changed paths (solve hand-off, residual at small B, dense Psi), then the floor
# probe and the ELB attribution
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_gibbs_dense_psi.py tests/test_gpu_gibbs_b3.py \
  tests/test_gpu_mirror.py tests/test_gpu_parity.py tests/test_gpu_sv_split.py tests/test_gpu_bh.py -x -v \
  --timeout 200 --timeout-method thread -s > gpurun_out/r06d_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probe_floor.py 20 > gpurun_out/r06d_floor.log 2>&1 || exit 1
bash tools/gpu/r06_c.sh
