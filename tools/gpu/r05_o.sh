#!/bin/bash
# k_sv_part on 4 workgroups x 4 waves per chain at B <= 32: SV split bit-identity and schedule tests,
# then the floor phases with the new layout and with 2 x 8 (CCMM_SV_NWG=2).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05o}
timeout -k 10 900 python -u -m pytest tests/test_gpu_sv_split.py tests/test_gpu_streams.py tests/test_gpu_bh.py \
  tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
CCMM_SV_NWG=2 timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_${TAG}_nwg2.json 2>> gpurun_out/floor_$TAG.err
