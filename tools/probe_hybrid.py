#!/usr/bin/env python
"""Kernel times of the hybrid-model sweep (mcmcVARhybridGibbs, K = 277) at B chains, as the
bench's hybrid line runs it: python tools/probe_hybrid.py [B] [sweeps] [option=value ...].  Timing-only ablation
switches (CCMM_CHOL_SKIP, CCMM_BIG_MASK, ...) are read by the library from the environment."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[3:])  # kernel options name=value
    import __graft_entry__ as ge
    pkg = ge.load_package()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, _, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    hm = pkg.model.build_hybrid(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, mpm, 0.25, e0, True)
    m = hm.var
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, store_capacity=steps + 1, seed=3,
                    model=pkg.MODEL_HYBRID, Ns=len(hm.ndxS), elbTmax=hm.elbT, elb_gibbsburn=100, elb=0.25,
                    options=opts or None)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(hm.ndxS, None)
    ch.set_elb_slot(0, hm.elbT0, hm.sNaN)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(1, store=True)
    ctx.synchronize()
    ch.profile(True)
    import time
    t0 = time.perf_counter()
    ch.sweep(steps, store=True)
    ctx.synchronize()
    el = time.perf_counter() - t0
    kt = ch.kernel_times()
    st = ch.get_status()
    print(json.dumps({"B": B, "options": opts, "ms_per_sweep": round(1e3 * el / steps, 3), "sweeps_per_s": round(B * steps / el, 1),
                      "flagged": int(np.count_nonzero(st & ~1)),
                      "kernel_ms_per_launch": {k: round(v[0] / v[1], 3) for k, v in kt.items() if v[1]}}))


if __name__ == "__main__":
    main()
