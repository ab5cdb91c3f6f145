#!/bin/bash
# k_sv_part over two workgroups per chain (B <= 128): bit-identity / parity tests and SV timing at small B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04w}
timeout -k 10 500 python -u -m pytest tests/test_gpu_sv_split.py tests/test_gpu_mirror.py tests/test_gpu_parity.py \
  tests/test_gpu_bh.py -x -v --timeout 200 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
for B in 1 16 64 128; do
  for w in 1 2; do
    echo "B=$B nwg=$w" >> gpurun_out/svsplit_$TAG.log
    CCMM_SV_NWG=$w timeout -k 10 120 python tools/kernel_times.py $B 2 6 >> gpurun_out/svsplit_$TAG.log 2>&1 || exit $?
  done
done
