#!/bin/bash
# k_chol_big phase attribution on the hybrid line (ablation build, timing only: CCMM_CHOL_SKIP bits
# 1 update, 2 factor, 4 panel, 8 tile factor+inverse, 16 inverse off-diagonal, 32 trailing tiles);
# k_gram_chol_lag with the tile factor+inverse skipped (CCMM_LAG_MODE 256) on the main line
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
export CCMM_LIB=$PWD/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for s in 0 1 2 4 8 16 32; do
  CCMM_CHOL_SKIP=$s timeout -k 10 120 python -u tools/probe_hybrid.py 256 2 > $O/skip$s.json 2>$O/skip$s.err || exit 1
  python -c "import json;d=json.load(open('$O/skip$s.json'));print($s, d['kernel_ms_per_launch']['k_chol_big'])"
done
for m in 0 256 1024; do
  CCMM_LAG_MODE=$m timeout -k 10 120 python -u tools/probe_main.py 256 5 > $O/lag$m.txt 2>&1 || exit 1
  echo "lag mode $m: $(grep k_gram_chol_lag $O/lag$m.txt)"
done
