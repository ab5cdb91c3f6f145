#!/bin/bash
# PMC summary of the main line (tools/probe_main.py 256 3 = bench.py's linear workload): one counter
# group per rocprofv3 pass (HBM FETCH / WRITE, MFMA, wave cycles), summarised by tools/pmc_summary.py into
# profiles/$TAG_pmc.json (read by bench.py for the roofline "traffic" and counter fields) and gpurun_out/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04t}
OUT=gpurun_out/pmc_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$R/$OUT/$name" -o run --output-format csv -- \
    python "$R/tools/probe_main.py" 256 3 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc $rc" >> "$OUT/passes.txt"
  return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass mfma SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
pass waves SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU &&
python tools/pmc_summary.py "profiles/${TAG}_pmc.json" "$OUT/fetch" "$OUT/write" "$OUT/mfma" "$OUT/waves" \
  > "$OUT/summary.log" 2>&1 && cp "profiles/${TAG}_pmc.json" "$OUT/"
