#!/bin/bash
# batched D-slab LDS fill in the lag kernels: bit-exact mirror tests, then main-line and floor kernel times
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mirror.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_main.py 256 10 > $O/main.txt 2>&1 && head -12 $O/main.txt && \
timeout -k 10 300 python -u tools/probe_floor.py 10 > $O/floor.json 2>$O/floor.err && tail -c 1500 $O/floor.json
