#!/bin/bash
# k_fcst register-resident coefficients: bit-identity + fcst tests, then predictive-line kernel stats
# for the (64,2) launch bound (default lib) and the (64) bound (libccmm_lb1.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=ccmmshadowratevar-code_amd/csrc
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py tests/test_gpu_fcst_hybrid.py \
  tests/test_gpu_batch_native.py > gpurun_out/r05am_tests.log 2>&1 &&
for v in lb2 lb1; do
  if [ $v = lb1 ]; then export CCMM_LIB=$R/$L/libccmm_lb1.so; fi
  rm -rf gpurun_out/prof_pred_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pred_$v" -o run --output-format csv -- \
    python "$R/bench.py" --no-cpu --bh-steps 0 --hy-steps 0 --oos-steps 0 --s120-steps 0 --girf-draws 0 \
    > gpurun_out/prof_pred_$v.json 2> gpurun_out/prof_pred_$v.err || exit 1
done
