"""Probe: the main line's linear sweeps (configs[1]: fredblockMD20, N = 20, p = 12, T = 750)
over B chains, Philox draws; prints per-kernel device times.  No result checks (for phase
ablations such as CCMM_SV_MODE).  Usage: python tools/probe_main.py [B] [sweeps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import __graft_entry__ as g

pkg = g.load_package()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nsw = int(sys.argv[2]) if len(sys.argv) > 2 else 5
d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
mpm = pkg.model.setMinnesotaMean(d["ncode"])
m = pkg.model.build_var(len(d["ydates"]), 12, 12, d["data"], d["ydates"], mpm, True)
ctx = pkg.Context(0)
ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False)
ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
st = pkg.model.initial_state(m, B)
ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
ch.sweep(2)
ctx.synchronize()
ch.profile(True)
t0 = time.perf_counter()
ch.sweep(nsw)
ctx.synchronize()
el = time.perf_counter() - t0
kt = ch.kernel_times()
print(f"B={B}: {1e3 * el / nsw:.3f} ms/sweep")
for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0]):
    if v[1]:
        print(f"  {k:18s} {v[0] / v[1]:9.4f} ms")
