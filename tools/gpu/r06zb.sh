#!/bin/bash
# k_elb_prep loads batched: BH / hybrid / shadow-rate parity, BH kernel times at 256 chains, floor
set -o pipefail
O=gpurun_out/r06zb; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bh.py tests/test_gpu_hybrid.py tests/test_gpu_shadowrate.py tests/test_gpu_elb_wavefront.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/kernel_times_bh.py 256 > $O/bh.txt 2>&1 && grep -E "elb_prep|ms" $O/bh.txt | head -5 && \
timeout -k 10 300 python -u tools/probe_floor.py 10 > $O/floor.json 2>$O/floor.err && python -c "
import json;d=json.load(open('$O/floor.json'))
for k in ('gibbs','ps','kept'):
  v=d.get(k,{}); print(k, v.get('ms_per_sweep'), v['kernel_ms_per_launch'].get('k_elb_prep'))"
