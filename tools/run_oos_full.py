#!/usr/bin/env python
"""The full quasi-real-time OOS run of goVARshadowrateBlockHybrid.m (BASELINE.json
configs[3]) on one GPU, end to end, as the reference driver sets it up (:34-160):
fredblockMD20-2022-09, ELB 0.25, p = 12, every jump-off after 2008-12 (164 vintages),
MCMCdraws = 1000 kept after 1000 burn-in sweeps, fcstNdraws = 10 * MCMCdraws, 48 horizons,
one chain per vintage; the ELB step Gibbs for m < 500 then 1000 PS proposals with Gibbs
fallback; the per-vintage post-processing of :318-480 (log scores, median / quantiles /
CRPS of the forecast paths and their cumulated form, PAI moments and quantiles,
shadow-rate vintages, max VAR root of every draw) and the QRT summary file of :641-669.

Writes a JSON summary (wall times of each phase, per-vintage log scores, acceptance counts,
the saved .mat varlist with shapes) to --out; the .mat file itself goes to --mat.

Run: python tools/run_oos_full.py [--draws 1000] [--out gpurun_out/oos_full.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--draws", type=int, default=1000)
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/oos_full.json")
    ap.add_argument("--mat", default="/tmp/fredblockMD20-2022-09-ELBblockhybrid-p12.mat")
    ap.add_argument("--no-maxlambda", action="store_true")
    args = ap.parse_args()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    S = pkg.samplers
    t_all = time.perf_counter()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    N = d["data"].shape[1]
    t0 = time.perf_counter()
    res = S.goVARshadowrateBlockHybrid_batch(
        d["data"], d["ydates"], ndxS, ndxO, mpm, MCMCdraws=args.draws, fcstNdraws=10 * args.draws,
        fcstNhorizons=48, ELBbound=0.25, nchains=args.chains, postprocess=True, cumcode=d["cumcode"],
        maxlambda=not args.no_maxlambda, progress=True, chunk=100)
    t_batch = time.perf_counter() - t0
    t0 = time.perf_counter()
    actual = ~np.isin(np.arange(N), ndxY)
    names = S.save_qrt_mat(args.mat, res, data=d["data"], ydates=d["ydates"], p=12, ncode=d["ncode"],
                           tcode=d["tcode"], cumcode=d["cumcode"], ndxSHADOWRATE=ndxS, ndxOTHERYIELDS=ndxO,
                           ELBbound=0.25, actualrateBlock=actual, datalabel="fredblockMD20-2022-09",
                           modellabel="ELBblockhybrid", MCMCdraws=args.draws, fcstNhorizons=48)
    t_save = time.perf_counter() - t0
    from scipy.io import loadmat, whosmat
    shapes = {n: list(s) for n, s, _ in whosmat(args.mat)}
    m = loadmat(args.mat, variable_names=["fcstYmvlogscore", "Tjumpoffs"])
    st = res["stats"]
    V = len(res["Tjumpoffs"])
    out = {
        "workload": f"configs[3]: goVARshadowrateBlockHybrid full OOS run, {V} vintages x {args.chains} chain(s), "
                    f"{args.draws} burn-in + {args.draws} kept sweeps each, fcstNdraws = {10 * args.draws}, "
                    "48 horizons, ELB 0.25 (Gibbs for m < 500, then 1000 PS proposals with Gibbs fallback), "
                    "per-vintage post-processing on the device, max VAR root on the host, QRT .mat written",
        "wall_s": {"total": round(time.perf_counter() - t_all, 2), "batch": round(t_batch, 2),
                   "setup": round(st["setup_s"], 2), "sampling_and_postprocess": round(st["run_s"], 2),
                   "save_mat": round(t_save, 2)},
        "sweeps": st["sweeps_local"],
        "sweeps_per_s": round(st["sweeps_local"] / st["run_s"], 1),
        "retries": st["retries"],
        "vintages": V,
        "Tjumpoffs": [int(t) for t in res["Tjumpoffs"]],
        "fcstYmvlogscore": [None if not np.isfinite(x) else round(float(x), 6) for x in res["fcstYmvlogscore"]],
        "fcstYmvlogscoreX": [None if not np.isfinite(x) else round(float(x), 6) for x in res["fcstYmvlogscoreX"]],
        "fcstYmvlogscoreI": [None if not np.isfinite(x) else round(float(x), 6) for x in res["fcstYmvlogscoreI"]],
        "countELBaccept": [int(x) for x in res["countELBaccept"]],
        "finite_logscores": int(np.isfinite(res["fcstYmvlogscore"]).sum()),
        "mat_file": os.path.basename(args.mat), "mat_bytes": os.path.getsize(args.mat),
        "mat_varlist": shapes,
        "mat_roundtrip_logscore_equal": bool(np.array_equal(np.ravel(m["fcstYmvlogscore"]),
                                                            np.ravel(res["fcstYmvlogscore"]), equal_nan=True)),
        "reference_varlist": "goVARshadowrateBlockHybrid.m:645-655 (data, ydates, p, Tjumpoffs, N, ncode, tcode, "
                             "cumcode, fcst*, fcstNhorizons, PAI*, shadowrate*, missingrate*, ndxSHADOWRATE, "
                             "ndxYIELDS, ndxOTHERYIELDS, ELBbound, ELBdummy, actualrateBlock, datalabel, modellabel, "
                             "doQuarterly, setQuantiles, MCMCdraws); doLoMem = true (:59) drops sumFFR* / VMA*",
    }
    if "drawsMaxVARroot" in res:
        mx = res["drawsMaxVARroot"]
        out["maxVARroot_median_first_last"] = [round(float(np.median(mx[:, 0])), 5),
                                               round(float(np.median(mx[:, -1])), 5)]
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("wall_s", "sweeps", "sweeps_per_s", "finite_logscores", "mat_bytes")}))


if __name__ == "__main__":
    main()
