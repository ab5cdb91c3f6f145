#!/bin/bash
# round-3 check 3: full GPU suite after the substitution solve and the wavefront ELB passes,
# kernel times (main line, BH with 1/4/8 passes in flight), full OOS run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s -rf \
  > gpurun_out/r03_check3_tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/probe_main.py 256 5 > gpurun_out/r03_probe_main.log 2>&1 || exit 1
for w in 1 4 8; do
  echo "waves $w" >> gpurun_out/r03_probe_bh.log
  CCMM_ELB_WAVES=$w timeout -k 10 120 python -u tools/kernel_times_bh.py 256 1 3 >> gpurun_out/r03_probe_bh.log 2>&1 || exit 1
done
OPENBLAS_NUM_THREADS=1 timeout -k 10 600 python -u tools/run_oos_full.py --no-maxlambda \
  --out gpurun_out/r03_oos_full.json > gpurun_out/r03_oos_full.log 2>&1
