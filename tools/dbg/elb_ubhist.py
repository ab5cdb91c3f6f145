#!/usr/bin/env python
"""Histogram of ub = (elb - mu) / sigma over the Gibbs draws of k_elb_gibbs_mp at the OOS floor (thisT = 762,
one chain; ablation build CCMM_LIB=.../libccmm_ablation.so with CCMM_ELB_MODE=4096).  Timing-free."""
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
    lib = ctypes.CDLL(os.environ["CCMM_LIB"])
    buf = (ctypes.c_ulonglong * 8)()
    ch.sweep(3, store=False)  # past the initial state
    ctx.synchronize()
    lib.ccmm_elb_ubhist(buf, 1)
    ch.sweep(steps, store=False)
    ctx.synchronize()
    lib.ccmm_elb_ubhist(buf, 0)
    h = list(buf[:7])
    names = ["ub>=9", "7-9", "5-7", "3-5", "1-3", "-1-1", "<-1"]
    tot = max(sum(h), 1)
    print(json.dumps({"draws": sum(h), "frac": {n: round(v / tot, 4) for n, v in zip(names, h)}}))
    ch.close()


if __name__ == "__main__":
    main()
