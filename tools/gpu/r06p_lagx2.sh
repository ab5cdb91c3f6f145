#!/bin/bash
# solve residual phase with 32 loads in flight; hybrid + S120 A/B of the lag twin
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hybrid.py tests/test_gpu_s120.py tests/test_gpu_mirror.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 > $O/hy.json 2>$O/hy.err && cat $O/hy.json && \
timeout -k 10 300 python -u tools/probe_s120_sweep.py 56 2 big_lagx=1 > $O/s120_on.txt 2>&1 && head -8 $O/s120_on.txt && \
timeout -k 10 300 python -u tools/probe_s120_sweep.py 56 2 big_lagx=0 > $O/s120_off.txt 2>&1 && head -8 $O/s120_off.txt
