#!/bin/bash
# GPU round script: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1" >> gpurun_out/steps.log; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || exit 2
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
step bench
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 4
step prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || exit 5
step done
