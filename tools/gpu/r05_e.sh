#!/bin/bash
# octet kernel back to the full draw (no per-step AS241 precompute), device PAI moments in ccmm_run_batch:
# ELB schedule bit-identity + batch parity, then the OOS lines (C = 1: measured full run + floor) and BH 1024.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_elb_wavefront.py tests/test_gpu_batch_native.py tests/test_gpu_oos.py \
  -x -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 900 python -u bench.py --no-cpu --steps 10 --no-fcst --bh-chains 256,1024 --hy-steps 0 --s120-steps 0 \
  --girf-draws 0 --oos-chains 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
