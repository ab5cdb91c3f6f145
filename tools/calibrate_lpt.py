#!/usr/bin/env python
"""Measure the per-vintage cost of the OOS batch (goVARshadowrateBlockHybrid.m:258, one chain per
vintage) on the GPU and fit the coefficients of distributed.unit_cost.

For every `stride`-th vintage (jump-offs after 2008-12) one chain runs alone in its own chain set
through the reference's three ELB phases (bench._oos_timed: Gibbs burn-in sweeps, PS burn-in
sweeps, kept sweeps with the predictive density); its full-run time is 500 Gibbs + 500 PS + 1000
kept sweeps at the measured rates.  Fit (non-negative least squares, seconds per full run):

    t = a T + c S(n_cens) + e n_cens,   S = ELB wavefront steps (distributed.elb_wavefront_steps)

Writes the measurements, the fit and its residuals as JSON.
Usage: calibrate_lpt.py OUT.json [stride] [steps]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402


def main(out, stride=12, steps=4):
    from scipy.optimize import nnls
    pkg = ge.load_package()
    S, dm = pkg.samplers, pkg.distributed
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p, H, Nd = 12, 48, 10
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    bench._OOS_NDXY[0] = ndxY
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    Tj = [int(t) for t in (np.flatnonzero(d["ydates"] > S.datenum(2008, 12, 1)) + 1)]
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    startELB = e0 + 1 + p
    ctx = pkg.Context(0)
    sel = sorted(set(list(range(0, len(Tj), stride)) + [len(Tj) - 1]))
    rows = []
    for v in sel:
        t0 = time.time()
        u = S._bh_units(d["data"], d["ydates"], [Tj[v]], p, 12, ndxS, ndxO, mpm, 0.25, e0, True, H)
        (fg, fb, fk), _, _, _, _ = bench._oos_timed(S, ctx, u, 1, np.array([v], np.uint32), steps,
                                                    lambda: ctx.synchronize(), H, Nd, False)
        nc = dm.censored_months(d["data"], ndxS, 0.25, startELB, Tj[v])
        full = (500 * fg + 500 * fb + 1000 * fk) / steps
        rows.append({"vintage": v, "thisT": Tj[v], "T": Tj[v] - p, "n_cens": nc,
                     "ms_gibbs": 1e3 * fg / steps, "ms_ps": 1e3 * fb / steps, "ms_kept": 1e3 * fk / steps,
                     "full_run_s": full})
        print(json.dumps(rows[-1]), f"({time.time() - t0:.1f}s)", flush=True)
    A = np.array([[r["T"], dm.elb_wavefront_steps(r["n_cens"]), r["n_cens"]] for r in rows], float)
    y = np.array([r["full_run_s"] for r in rows])
    coef, _ = nnls(A, y)
    fit = A @ coef
    res = {"note": "per-vintage full-run seconds (500 Gibbs + 500 PS + 1000 kept sweeps, one chain alone); "
                   "fit t = a T + c S(n_cens) + e n_cens (NNLS)",
           "coef": {"a_per_T": coef[0], "c_per_elb_step": coef[1], "e_per_cens_month": coef[2]},
           "max_rel_residual": float(np.max(np.abs(fit - y) / y)), "rows": rows,
           "fit_s": fit.tolist()}
    Path(out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res["coef"]), "max rel residual", res["max_rel_residual"])


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
