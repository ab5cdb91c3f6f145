#!/bin/bash
# k_fcst<20> (16-byte ring reads): bit-identity + fcst tests, then predictive-line kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05an}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py tests/test_gpu_fcst_hybrid.py \
  tests/test_gpu_batch_native.py > gpurun_out/${TAG}_tests.log 2>&1 &&
rm -rf gpurun_out/prof_pred_$TAG &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pred_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 \
  > gpurun_out/prof_pred_$TAG.json 2> gpurun_out/prof_pred_$TAG.err
