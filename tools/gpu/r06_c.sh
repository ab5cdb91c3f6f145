#!/bin/bash
# round 6: ELB month-latency attribution at the OOS floor (ablation build, timing only), and the octet
# kernel at B = 1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r06c_floor_abl.log
for cfg in "elb_oct=2" "elb_waves=4 elb_parts=1" "elb_waves=1 elb_parts=1"; do
  echo "== product $cfg" >> $O
  timeout -k 10 200 python -u tools/probe_floor.py 10 $cfg >> $O 2>&1 || exit 1
done
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 1 512 256 2 128 769; do
  echo "== mode $m" >> $O
  CCMM_ELB_MODE=$m timeout -k 10 200 python -u tools/probe_floor.py 10 elb_parts=1 >> $O 2>&1 || exit 1
done
