#!/usr/bin/env python
"""Kernel times of the OOS per-rank floor (bench.py bench_oos floor=True: the longest vintage,
thisT = 762, 1 chain) for each ELB phase (Gibbs burn-in, PS burn-in, kept sweeps):
python tools/probe_floor.py [steps] [option=value ...] (kernel options, ccmm_set_option).  Timing-only.
Without wall-clock profiling events ("noprof" as an option) the sweep time is the event-free wall time."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
    noprof = False
    for kv in sys.argv[2:]:
        if kv == "noprof":
            noprof = True
            continue
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ch, _, _ = S._bh_chain_set(ctx, u1, 1, seed=1012023, ids=np.array([0], np.uint32),
                               store_capacity=steps + 1, gibbsburn=100, ELBbound=0.25, ndxYIELDS=ndxY,
                               fcstNhorizons=48, Nd=10)
    ch.set_elb_ps(1000, 2 + steps)
    ch.sweep(1, store=True)
    ch.get_fcst()
    ch.get_draws()
    out = {}
    for name, store in (("gibbs", False), ("ps", False), ("kept", True)):
        ch.profile(not noprof)
        ctx.synchronize()
        t0 = time.perf_counter()
        ch.sweep(steps, store=store)
        ctx.synchronize()
        el = time.perf_counter() - t0
        kt = ch.kernel_times()
        ch.profile(False)
        out[name] = {"ms_per_sweep": round(1e3 * el / steps, 3),
                     "kernel_ms_per_launch": {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]},
                     "launches_per_sweep": {k: round(v[1] / steps, 2) for k, v in kt.items() if v[1]}}
        if store:
            ch.get_draws()
            ch.get_fcst()
    out["status"] = int(np.count_nonzero(ch.get_status()))
    ch.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
