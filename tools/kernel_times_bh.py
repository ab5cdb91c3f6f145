#!/usr/bin/env python
"""Developer tool: per-kernel device time of the block-hybrid sweep (real data,
ELB = 0.25, 2022-08 jump-off, B chains), for A/B and ablation runs driven by
CCMM_* environment variables (CCMM_ELB_MODE, CCMM_LAG_MODE, ...).  Does not
check results (ablation builds produce invalid draws).
Usage: kernel_times_bh.py [B] [warmup] [steps] [nproposals (0: Gibbs every sweep)]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402


def main(B=256, warm=1, steps=3, nproposals=0):
    pkg = ge.load_package()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    bm = pkg.model.build_bh(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, ndxO, mpm, 0.25, e0)
    m = bm.var
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, seed=1, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=100, elb=0.25)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm.ndxS, bm.actual_block)
    ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
    if nproposals:                       # PS proposals with the Gibbs fallback at every sweep
        ch.set_elb_ps(nproposals, 1)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    try:
        ch.sweep(warm)
    except RuntimeError as e:
        print("warmup:", e)
    ch.profile(True)
    t0 = time.perf_counter()
    try:
        ch.sweep(steps)
    except RuntimeError as e:
        print("sweep:", e)
    ctx.synchronize()
    el = time.perf_counter() - t0
    kt = {k: round(v[0] / v[1], 4) for k, v in ch.kernel_times().items() if v[1]}
    print(json.dumps({"ms_per_sweep": round(1e3 * el / steps, 3), "kernels": kt}))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
