"""Debug: CTAsys toy case through the generic and the large CTA path, per-equation error."""
import os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import numpy as np
import __graft_entry__ as g
from oracle import ccmm_oracle as O
from helpers import random_state, toy_setup
pkg = g.load_package()
ctx = pkg.Context(0)
os.environ["CCMM_FORCE_BIG"] = "1"
fred = O.load_fred_csv(Path(__file__).resolve().parents[1] / "tests/golden/data/fredblockMD20-2022-09.csv")
mpm = O.set_minnesota_mean(fred["ncode"])
sr = O.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
s0 = random_state(O, sr, seed=5)
r0 = np.random.default_rng(4)
g0, _ = ctx.cta(sr.Y, sr.X, s0["A"][..., None], s0["sqrtht"][..., None], sr.iVdiag, sr.iVb, s0["PAI"][..., None], r0.standard_normal((sr.K, sr.N))[..., None])
print("real done", np.isfinite(g0).all())
del os.environ["CCMM_FORCE_BIG"]
su = toy_setup(O, N=5, p=3, Tobs=90, seed=2)
rng = np.random.default_rng(9)
XX = np.repeat(su.X[:, :, None], su.N, axis=2)
XX[:, 1:, 3:] += 0.1 * rng.standard_normal((su.T, su.K - 1, su.N - 3))
sts = [random_state(O, su, seed=8 + c) for c in range(2)]
zs = [rng.standard_normal((su.K, su.N)) for _ in range(2)]
P0 = [s["PAI"] + 0.01 * rng.standard_normal(s["PAI"].shape) for s in sts]
for force in (1, 0, 1):
    if force:
        os.environ["CCMM_FORCE_BIG"] = "1"
    elif "CCMM_FORCE_BIG" in os.environ:
        del os.environ["CCMM_FORCE_BIG"]
    got, status = ctx.cta(su.Y, XX, np.stack([s["A"] for s in sts], -1), np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb, np.stack(P0, -1), np.stack(zs, -1))
    for c in range(2):
        want, _, sd = O.cta_sys(su.Y, XX, su.N, su.K, su.T, sts[c]["A"], sts[c]["sqrtht"], su.iVdiag, su.iVb, P0[c], zs[c], return_sd=True)
        e = np.abs(got[..., c] - want) / np.maximum(np.abs(want), sd)
        print("force", force, "chain", c, "status", status, "err per eq", e.max(axis=0))
