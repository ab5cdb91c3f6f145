#!/bin/bash
# k_fcst split (paths per (draw, chain) + k_fcst_scores): forecast parity tests, the batch / OOS tests
# that read forecasts, then the OOS floor phases (default library and the FCST_MODE ablations).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05b}
ABL=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_fcst.py tests/test_gpu_fcst_chain.py tests/test_gpu_fcst_hybrid.py \
  tests/test_gpu_batch_native.py tests/test_gpu_shadowrate_batch.py -x -v --timeout 200 --timeout-method thread -s -rf \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_$TAG.json 2> gpurun_out/floor_$TAG.err &&
for m in "FCST_MODE=1" "FCST_MODE=2"; do
  env CCMM_LIB=$ABL CCMM_$m timeout -k 10 120 python tools/probe_floor.py 10 > gpurun_out/floor_${TAG}_$m.json \
    2> gpurun_out/floor_${TAG}_$m.err || exit $?
done
