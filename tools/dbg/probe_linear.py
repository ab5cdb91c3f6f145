#!/usr/bin/env python
"""Per-kernel device times of the linear-model sweep (configs[1]: fredblockMD20, N = 20, p = 12,
T = 750, B chains): python tools/dbg/probe_linear.py [B] [steps].  Timing-only; CCMM_* switches
(and CCMM_LIB) are read from the env; chain status is reported, not enforced."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import __graft_entry__ as ge
    pkg = ge.load_package()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    m = pkg.model.build_var(len(d["ydates"]), 12, 12, d["data"], d["ydates"], mpm, True)
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, seed=5)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(1)
    ctx.synchronize()
    ch.profile(True)
    ch.sweep(steps)
    ctx.synchronize()
    kt = ch.kernel_times()
    out = {"B": B, "kernel_ms_per_launch": {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]},
           "status_nonzero": int(np.count_nonzero(ch.get_status()))}
    ch.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
