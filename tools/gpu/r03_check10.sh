#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_hybrid.py tests/test_gpu_bign.py \
  tests/test_gpu_s120.py -v --timeout 300 --timeout-method thread -s -rf > gpurun_out/r03_check10_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for m in 0 2 8; do
  echo "skip $m" >> gpurun_out/r03_probe_hybrid10.log
  CCMM_CHOL_SKIP=$m timeout -k 10 120 python -u tools/probe_hybrid.py 256 3 >> gpurun_out/r03_probe_hybrid10.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --warmup 1 --bh-steps 0 --hy-steps 0 --oos-steps 0 --girf-draws 0 \
  --no-fcst --s120-steps 2 > gpurun_out/r03_s120_bench10.json 2> gpurun_out/r03_s120_bench10.err
