#!/bin/bash
# Instruction-issue counters of the block-hybrid sweep's per-chain kernels (k_elb_gibbs, k_sv_part,
# k_cta_solve_lag, ...): is a kernel VALU-issue-bound (SQ_INSTS_VALU x 4 cycles per wave64 instruction
# ~ the SIMDs' cycles) or latency-bound?  One counter group per rocprofv3 pass, each pass under its
# own time limit; the first pass that faults, aborts or times out ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
B=${B:-256}
OUT=gpurun_out/pmc_issue_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run --output-format csv -- \
  python "$R/tools/kernel_times_bh.py" "$B" 1 2 > "$OUT/trace.log" 2>&1 || exit $?
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$R/$OUT/$name" -o run --output-format csv -- \
    python "$R/tools/kernel_times_bh.py" "$B" 1 2 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc $rc" >> "$OUT/passes.txt"
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
pass issue SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
pass active SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
python tools/pmc_summary.py "$OUT/summary.json" "$OUT/issue" "$OUT/active" > "$OUT/summary.log" 2>&1
exit 0
