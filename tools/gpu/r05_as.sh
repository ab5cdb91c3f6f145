#!/bin/bash
# k_chol_big panel prefetch: large-path tests, hybrid kernel stats, then the solve_big phase ablation
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05as}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_big.py tests/test_gpu_hybrid.py tests/test_gpu_bign.py > gpurun_out/${TAG}_tests.log 2>&1 &&
rm -rf gpurun_out/prof_hy_$TAG &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_hy_$TAG" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu --steps 1 --warmup 0 --no-fcst --bh-steps 0 --hy-steps 3 --hy-chains 256 \
  --oos-steps 0 --oos-full-draws 0 --s120-steps 0 --girf-draws 0 \
  > gpurun_out/prof_hy_$TAG.json 2> gpurun_out/prof_hy_$TAG.err || exit 1
bash tools/gpu/r05_ar.sh
