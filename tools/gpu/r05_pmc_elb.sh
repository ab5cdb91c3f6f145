#!/bin/bash
# Issue / wait counters of the per-chain kernels: the B = 256 block-hybrid sweep (the bench's ELB
# report: profiles/*pmc_issue*.json) and the OOS floor (one chain, tools/probe_floor.py).  One counter
# group per rocprofv3 pass, each pass under its own time limit; a failing pass ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r05}
pass() {
  local out=$1 name=$2; shift 2
  local cmd=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$R/$out/$name" -o run --output-format csv -- $cmd > "$out/$name.log" 2>&1
  local rc=$?
  echo "pass $out/$name rc $rc" >> gpurun_out/pmc_passes_$TAG.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
for W in bh256 floor; do
  OUT=gpurun_out/pmc_issue_${TAG}_$W
  rm -rf "$OUT"; mkdir -p "$OUT"
  if [ $W = bh256 ]; then CMD="python $R/tools/kernel_times_bh.py 256 1 2"; else CMD="python $R/tools/probe_floor.py 3"; fi
  pass $OUT issue "$CMD" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
  pass $OUT active "$CMD" SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE &&
  python tools/pmc_summary.py "$OUT/summary.json" "$OUT/issue" "$OUT/active" > "$OUT/summary.log" 2>&1 || exit $?
done
