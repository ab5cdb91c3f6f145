#!/bin/bash
# GPU round script: parity tests, bench, rocprofv3 kernel stats.  Each GPU step time-limited.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -s > gpurun_out/tests.log 2>&1
echo "tests exit=$?" >> gpurun_out/tests.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1 || exit 4
