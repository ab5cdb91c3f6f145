#!/usr/bin/env python
"""Summarise rocprofv3 --pmc counter CSVs into per-kernel HBM bytes per launch.

Usage: pmc_summary.py OUT.json DIR [DIR ...]
Each DIR holds the output of one `rocprofv3 --pmc <counters> -d DIR -o run
--output-format csv` pass (one counter group per pass, MI355X_MICROARCH.md
"HBM").  Corrections (same guide): FETCH_SIZE reports half the bytes of a wide
coalesced read on gfx950, so it is doubled; WRITE_SIZE is taken as is.  Both
counters are in KiB.  Writes {kernel: {counter: mean per launch, ..., "launches": n}}.
MFMA pass (SQ_INSTS_VALU_MFMA_MOPS_F64, SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...):
"mfma_f64_flop" = 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 (the counter's unit, as rocprof-compute's
FLOP derivation), "mfma_busy_frac" = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs
x 4 SIMDs) (GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md "DVFS"), and
"clock_ghz_est" = GRBM_GUI_ACTIVE / 8 / launch time when the kernel trace gives a duration.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    name = name.split("(")[0]
    for pre in ("void ", "ccmm::"):
        name = name.replace(pre, "")
    return name.split("<")[0].strip()


def main(out, *dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in Path(d).rglob("*counter_collection.csv"):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    c = row.get("Counter_Name", "")
                    try:
                        v = float(row.get("Counter_Value", "nan"))
                    except ValueError:
                        continue
                    acc[k][(c, row.get("Dispatch_Id", ""))].append(v)
    res = {}
    for k, cv in acc.items():
        per = defaultdict(list)
        for (c, _disp), vals in cv.items():
            per[c].append(sum(vals))  # sum over XCD/instance rows of one dispatch
        r = {}
        for c, vals in per.items():
            mean = sum(vals) / len(vals)
            r[c] = mean
            r["launches_" + c] = len(vals)
            if c == "FETCH_SIZE":
                r["hbm_read_bytes"] = 2.0 * mean * 1024.0
            elif c == "WRITE_SIZE":
                r["hbm_write_bytes"] = mean * 1024.0
        if "hbm_read_bytes" in r and "hbm_write_bytes" in r:
            r["hbm_bytes"] = r["hbm_read_bytes"] + r["hbm_write_bytes"]
        if "SQ_INSTS_VALU_MFMA_MOPS_F64" in r:
            r["mfma_f64_flop"] = 512.0 * r["SQ_INSTS_VALU_MFMA_MOPS_F64"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r and r.get("GRBM_GUI_ACTIVE"):
            r["mfma_busy_frac"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / (r["GRBM_GUI_ACTIVE"] / 8.0 * 256 * 4)
        if "SQ_INSTS_VALU" in r and r.get("GRBM_GUI_ACTIVE"):
            # VALU issue: a wave64 VALU instruction holds its SIMD for 4 cycles (16 lanes per cycle; FP64
            # FMA is full rate on gfx950), over every SIMD cycle of the chip while the kernel runs
            r["valu_issue_frac"] = 4.0 * r["SQ_INSTS_VALU"] / (r["GRBM_GUI_ACTIVE"] / 8.0 * 256 * 4)
        res[k] = r
    Path(out).write_text(json.dumps(res, indent=1, sort_keys=True))
    for k in sorted(res):
        print(k, {c: round(v, 1) for c, v in res[k].items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
