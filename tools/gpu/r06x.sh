#!/bin/bash
# staged lag twin in k_cta_solve_big: hybrid + large-path parity (bit-exact mirror, twin identity), timing
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hybrid.py tests/test_gpu_bh.py::test_bh_large_path_lag_twin_bit_identical tests/test_gpu_s120.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 > $O/hy.json 2>$O/hy.err && cat $O/hy.json
