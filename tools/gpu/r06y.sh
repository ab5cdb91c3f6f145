#!/bin/bash
# batched LDS staging in k_phi / k_astep_w: parity, main-line and floor kernel times, BH line probe
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_astep_forms.py tests/test_gpu_mirror.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_main.py 256 10 > $O/main.txt 2>&1 && head -7 $O/main.txt && \
timeout -k 10 300 python -u tools/probe_floor.py 10 > $O/floor.json 2>$O/floor.err && python -c "
import json;d=json.load(open('$O/floor.json'))
for k in ('gibbs','ps','kept'):
  v=d.get(k,{}); print(k, v.get('ms_per_sweep'), {x:v['kernel_ms_per_launch'].get(x) for x in ('k_phi','k_astep')})"
