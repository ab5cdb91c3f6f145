#!/usr/bin/env python
"""Developer probe: the linear main-line workload (configs[1], N = 20, p = 12, B chains) run
as G chain groups on G HIP streams (one context each, one host thread per group), so the
per-chain sequential kernels of one group (CTA solve, SV, A-step) can overlap the MFMA
Gram/Cholesky of another.  Prints ms per step (all B chains swept once) per G.
Usage: probe_groups.py [B] [steps] [G,G,...] [lock]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402


def run(pkg, d, m, B, G, steps, lock):
    ctx0 = pkg.Context(0)
    ctxs = [ctx0] + [pkg.Context(0) for _ in range(G - 1)]
    Bg = B // G
    chs = []
    for g, cx in enumerate(ctxs):
        ch = pkg.Chains(cx, N=m.N, p=12, T=m.T, B=Bg, crn=False, store_capacity=steps + 3, seed=1012023)
        ch.set_rng_ids(np.arange(g * Bg, (g + 1) * Bg, dtype=np.uint32))
        if lock and G > 1:
            ch.set_mfma_lock(lock)
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        st = pkg.model.initial_state(m, Bg)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        chs.append(ch)
    bench._in_threads([lambda c=c: c.sweep(3, store=True) for c in chs])
    for cx in ctxs:
        cx.synchronize()
    t0 = time.perf_counter()
    bench._in_threads([lambda c=c: c.sweep(steps, store=True) for c in chs])
    for cx in ctxs:
        cx.synchronize()
    el = time.perf_counter() - t0
    for c in chs:
        c.close()
    return 1e3 * el / steps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    Gs = [int(g) for g in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
    lock = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    pkg = ge.load_package()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    m = pkg.model.build_var(len(d["ydates"]), 12, 12, d["data"], d["ydates"], mpm, True)
    for G in Gs:
        ms = run(pkg, d, m, B, G, steps, lock)
        print(json.dumps({"B": B, "G": G, "lock": lock, "ms_per_step": round(ms, 3),
                          "sweeps_per_s": round(B / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
