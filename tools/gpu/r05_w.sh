#!/bin/bash
# LDS counters of the floor kernels (one chain): bank / address conflicts and LDS issue of the solve
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds_r05w; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/$OUT/lds -o run --output-format csv \
  -- python $R/tools/probe_floor.py 3 > $OUT/lds.log 2>&1 &&
python tools/pmc_summary.py $OUT/summary.json $OUT/lds > $OUT/summary.log 2>&1
