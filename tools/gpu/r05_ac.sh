#!/bin/bash
# MFMA / LDS counters of k_gram_chol_lag on the main line (linear, 256 chains): full kernel and SYRK
# only (CCMM_LAG_MODE=2, ablation build, timing only); one counter group per pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/pmc_gram_r05ac; rm -rf $OUT; mkdir -p $OUT
export CCMM_LIB=$R/ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so
for m in 0 2; do
  CCMM_LAG_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/$OUT/m$m -o run --output-format csv \
    -- python $R/tools/dbg/probe_linear.py 256 2 > $OUT/m$m.log 2>&1 || exit $?
  CCMM_LAG_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $R/$OUT/v$m -o run --output-format csv \
    -- python $R/tools/dbg/probe_linear.py 256 2 > $OUT/v$m.log 2>&1 || exit $?
  python tools/pmc_summary.py $OUT/summary_m$m.json $OUT/m$m $OUT/v$m > $OUT/summary_m$m.log 2>&1
done
