#!/bin/bash
# ELB Gibbs iteration: BH/hybrid/vintage parity tests, then block-hybrid kernel timings
# for each CCMM_ELB_MODE in EMODES (timing-only ablations after mode 0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; : > gpurun_out/elb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bh.py tests/test_gpu_hybrid.py tests/test_gpu_vintages.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests exit=$rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
for m in ${EMODES:-0}; do
  echo "elb mode=$m" >> gpurun_out/elb.log
  CCMM_ELB_MODE=$m timeout -k 10 120 python tools/kernel_times_bh.py 256 1 3 >> gpurun_out/elb.log 2>&1 || exit 2
done
