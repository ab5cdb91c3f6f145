"""Probe: full block-hybrid sweeps at the S120 shape (N = 120, p = 12, K = 1441, T = 750) on
the synthetic panel, B chains, Philox draws; prints the per-kernel device times.  No result
checks (phase ablations such as CCMM_SV_SKIP produce meaningless draws).
Usage: python tools/probe_s120_sweep.py [B] [sweeps] [option=value ...]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np

import __graft_entry__ as g

pkg = g.load_package()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
nsw = int(sys.argv[2]) if len(sys.argv) > 2 else 2
opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[3:])  # kernel options name=value
p = 12
d = pkg.synthetic.s120()
ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
bm = pkg.model.build_bh(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, ndxO,
                        np.ones(d["data"].shape[1]), 0.25, e0, True)
m = bm.var
ctx = pkg.Context(0)
ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=100, elb=0.25, options=opts or None)
ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
ch.set_elb_model(bm.ndxS, bm.actual_block)
ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
st = pkg.model.initial_state(m, B)
ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
ch.sweep(1)
ctx.synchronize()
ch.profile(True)
t0 = time.perf_counter()
ch.sweep(nsw)
ctx.synchronize()
el = time.perf_counter() - t0
kt = ch.kernel_times()
print(f"B={B} {opts}: {1e3 * el / nsw:.1f} ms/sweep")
for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0]):
    if v[1]:
        print(f"  {k:18s} {v[0] / v[1]:9.3f} ms")
