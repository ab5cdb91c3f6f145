#!/bin/bash
# round-3 measurement, part 2: PMC passes over the main line (HBM bytes, MFMA busy), then the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03f}
run_pass() {
  local name=$1; shift
  rm -rf "gpurun_out/pmc_${TAG}_$name"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$R/gpurun_out/pmc_${TAG}_$name" -o run --output-format csv \
    -- python "$R/tools/probe_main.py" 256 3 > "gpurun_out/pmc_${TAG}_$name.log" 2>&1
}
run_pass mfma SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
