#!/bin/bash
# quick GPU iteration: parity tests + bench (no CPU baseline, no rocprof)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -s -x > gpurun_out/tests.log 2>&1
echo "tests exit=$?" >> gpurun_out/tests.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench exit=$?" >> gpurun_out/bench.err
