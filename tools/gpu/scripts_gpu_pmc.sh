#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) over the probe command in $PROBE:
#   PROBE="tools/probe_main.py 256 3" scripts_gpu_pmc.sh <tag>
# each pass leaves its counter_collection.csv under gpurun_out/pmc_<tag>_<pass>/
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
run_pass() {
  local name=$1; shift
  rm -rf "gpurun_out/pmc_${TAG}_$name"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$R/gpurun_out/pmc_${TAG}_$name" -o run --output-format csv -- python $PROBE > "gpurun_out/pmc_${TAG}_$name.log" 2>&1
}
run_pass mfma SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE
