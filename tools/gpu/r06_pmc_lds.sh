#!/bin/bash
# LDS counters per kernel at the OOS floor (probe_floor, B = 1) and on the main line (probe_main, B = 256)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06i}
OUT=gpurun_out/pmclds_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d "$R/$OUT/floor" -o run --output-format csv -- python "$R/tools/probe_floor.py" 3 > "$OUT/floor.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d "$R/$OUT/main" -o run --output-format csv -- python "$R/tools/probe_main.py" 256 3 > "$OUT/main.log" 2>&1 &&
python tools/pmc_summary.py "$OUT/floor.json" "$OUT/floor" > "$OUT/s1.log" 2>&1 &&
python tools/pmc_summary.py "$OUT/main.json" "$OUT/main" > "$OUT/s2.log" 2>&1
