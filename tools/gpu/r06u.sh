#!/bin/bash
# k_chol_big diagonal-block load batched: hybrid parity + timing; k_sv_part phase split (ablation build)
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hybrid.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/probe_hybrid.py 256 3 > $O/hy.json 2>$O/hy.err && cat $O/hy.json || exit 1
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 1 2 4 8 16 64; do
  CCMM_SV_MODE=$m timeout -k 10 120 python -u tools/probe_main.py 256 5 > $O/sv$m.txt 2>&1 || exit 1
  echo "sv mode $m: $(grep k_sv_part $O/sv$m.txt)"
done
