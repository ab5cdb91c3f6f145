#!/bin/bash
# bench.py default run (all lines incl. the measured full configs[3] run) + the batch PSRF test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_native.py -x -v --timeout 200 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
