#!/bin/bash
# k_chol_big panel bursts double-buffered: hybrid parity + timing, S120 timing
set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hybrid.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 > $O/hy.json 2>$O/hy.err && cat $O/hy.json && \
timeout -k 10 300 python -u tools/probe_s120_sweep.py 56 2 > $O/s120.txt 2>&1 && head -5 $O/s120.txt
