#!/bin/bash
# k_gram_chol_lag tile inverse fused into the factor: mirror bit-exact, main-line kernel times
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mirror.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_main.py 256 10 > $O/main.txt 2>&1 && head -5 $O/main.txt
