#!/bin/bash
# GPU iteration for the block-hybrid path: BH parity tests first, then the whole GPU suite.
# Stops at the first failing step (no GPU work after a failure).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_bh.py -q -s -x > gpurun_out/bh.log 2>&1
rc=$?; echo "bh exit=$rc" >> gpurun_out/bh.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1
rc=$?; echo "tests exit=$rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
