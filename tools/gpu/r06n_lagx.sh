#!/bin/bash
# Large path reading the lag twin of X (option big_lagx): parity tests, then hybrid A/B timings
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hybrid.py tests/test_gpu_s120.py tests/test_gpu_mirror.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 big_lagx=1 > $O/hy_on.json 2>$O/hy_on.err && \
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 big_lagx=0 > $O/hy_off.json 2>$O/hy_off.err && \
cat $O/hy_on.json $O/hy_off.json
