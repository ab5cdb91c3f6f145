#!/usr/bin/env python
"""Phase attribution of k_astep_w and k_cta_solve_lag at the OOS floor (thisT = 762, one chain;
ablation build, CCMM_LIB=.../libccmm_ablation.so): mean shader-clock cycles per launch of the A-step's
stage-E, Gram, factor + solves, invA and logy2, and of the solve's v_t, X'v (+ swap), forward,
backward and residual phases, beside the kernels' event times."""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import __graft_entry__ as ge
    pkg = ge.load_package()
    S = pkg.samplers
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    Tj = [int(t) for t in (np.flatnonzero(d["ydates"] > S.datenum(2008, 12, 1)) + 1)]
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    u1 = S._bh_units(d["data"], d["ydates"], [Tj[-1]], p, 12, ndxS, ndxO, mpm, 0.25, e0, True, 48)
    ctx = pkg.Context(0)
    ch, _, _ = S._bh_chain_set(ctx, u1, 1, seed=1012023, ids=np.array([0], np.uint32),
                               store_capacity=steps + 1, gibbsburn=100, ELBbound=0.25, ndxYIELDS=ndxY,
                               fcstNhorizons=48, Nd=10)
    ch.set_elb_ps(1000, 2 + steps)
    lib = ctypes.CDLL(os.environ["CCMM_LIB"])
    buf = (ctypes.c_ulonglong * 8)()
    sbuf = (ctypes.c_ulonglong * 8)()
    ch.sweep(1, store=False)
    ctx.synchronize()
    lib.ccmm_astep_prof(buf, 1)
    lib.ccmm_solve_prof(sbuf, 1)
    ch.profile(True)
    ch.sweep(steps, store=False)
    ctx.synchronize()
    kt = ch.kernel_times()
    lib.ccmm_astep_prof(buf, 0)
    lib.ccmm_solve_prof(sbuf, 0)
    a = np.array(buf[:], dtype=np.float64)
    n = max(a[5], 1)
    out = {"astep_ms": round(kt["k_astep"][0] / kt["k_astep"][1], 4), "launches": int(a[5])}
    out.update({k: round(a[i] / n) for i, k in enumerate(("stage", "gram", "factor", "inva", "logy2"))})
    b = np.array(sbuf[:], dtype=np.float64)
    n = max(b[5], 1)
    out["solve_ms"] = round(kt["k_cta_solve_lag"][0] / kt["k_cta_solve_lag"][1], 4)
    out["solve_cycles_per_launch"] = {k: round(b[i] / n) for i, k in
                                      enumerate(("v_t", "xv_swap", "forward", "backward", "residual"))}
    out["solve_cycles_per_launch"]["xv_only"] = round(b[6] / n)
    ch.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
