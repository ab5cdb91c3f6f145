#!/bin/bash
# k_cta_solve_big phase attribution on the hybrid line (ablation build, timing only: CCMM_SOLVE_SKIP
# bits 1 v/U, 2 X'v, 4 forward, 8 backward, 16 residual; draws invalid)
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for s in 0 1 2 4 8 16; do
  CCMM_SOLVE_SKIP=$s timeout -k 10 120 python -u tools/probe_hybrid.py 256 2 > $O/skip$s.json 2>$O/skip$s.err || exit 1
  python -c "import json;d=json.load(open('$O/skip$s.json'));print($s, d['kernel_ms_per_launch']['k_cta_solve_big'], d['kernel_ms_per_launch']['k_chol_big'])"
done
