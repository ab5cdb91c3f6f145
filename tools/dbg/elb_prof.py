#!/usr/bin/env python
"""Cycle attribution of the ASYNC ELB wavefront kernel at the OOS floor (thisT = 762, one chain):
needs the ablation build (CCMM_LIB=.../libccmm_ablation.so) and CCMM_ELB_MODE with bit 64 set.
Prints, per wave, the mean shader-clock cycles per month spent waiting for the predecessor pass,
in the neighbour sums, in the draws and in the store/publish tail."""
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
    buf = (ctypes.c_ulonglong * 48)()
    ch.sweep(1, store=False)
    ctx.synchronize()
    lib.ccmm_elb_prof(buf, 1)
    ch.profile(True)
    ch.sweep(steps, store=False)
    ctx.synchronize()
    kt = ch.kernel_times()
    lib.ccmm_elb_prof(buf, 0)
    a = np.array(buf[:], dtype=np.float64).reshape(8, 6)
    out = {"elb_ms": round(kt["k_elb_gibbs"][0] / kt["k_elb_gibbs"][1], 4), "mode": os.environ.get("CCMM_ELB_MODE")}
    for w in range(8):
        m = max(a[w, 4], 1)
        out[f"wave{w}"] = {"months": int(a[w, 4]), "wait": round(a[w, 0] / m), "sums": round(a[w, 1] / m),
                           "draws": round(a[w, 2] / m), "tail": round(a[w, 3] / m)}
    tot = a[:, :4].sum(0) / max(a[:, 4].sum(), 1)
    out["mean_cycles_per_month"] = dict(zip(("wait", "sums", "draws", "tail"), [round(x) for x in tot]))
    ch.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
