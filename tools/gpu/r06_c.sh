#!/bin/bash
# round 6: ELB month-latency attribution at the OOS floor (ablation build, timing only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
O=gpurun_out/r06c_floor_abl.log
for m in 0 1 512 256 2 128 769; do
  for cfg in "elb_parts=1" "elb_parts=1 elb_waves=4"; do
    echo "== mode $m $cfg" >> $O
    CCMM_ELB_MODE=$m timeout -k 10 200 python -u tools/probe_floor.py 10 $cfg >> $O 2>&1 || exit 1
  done
done
