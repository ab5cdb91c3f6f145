"""Debug: posterior sqrtht means of the toy linear model on the device, Philox vs CRN (numpy
normals), B chains, against the oracle run on the same CRN for chain 0."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np

import __graft_entry__ as ge
from helpers import crn_flat, toy_setup
from oracle import ccmm_oracle as oracle

pkg = ge.load_package()
ctx = pkg.Context(0)
su = toy_setup(oracle, N=4, p=2, Tobs=122, seed=11)
st0 = oracle.init_state(su)


def run(B, crn, nsw, keep):
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=crn, store_capacity=keep, seed=777)
    ch.set_data(0, su.Y, su.X, su.iVdiag, su.iVb, su.sPHI, su.Vol_0mean, su.Vol_0vcvsqrt)
    ch.set_state(*[np.repeat(st0[k][..., None], B, axis=-1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    crns = None
    if crn:
        rng = np.random.default_rng(3)
        crns = [[oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI) for _ in range(nsw)] for _ in range(B)]
        flat = np.stack([np.stack([crn_flat(oracle, crns[c][m], su) for m in range(nsw - keep)], -1)
                         for c in range(B)], -1)
        ch.sweep(nsw - keep, crn=flat)
        flat = np.stack([np.stack([crn_flat(oracle, crns[c][m], su) for m in range(nsw - keep, nsw)], -1)
                         for c in range(B)], -1)
        ch.sweep(keep, crn=flat, store=True)
    else:
        ch.sweep(nsw - keep)
        ch.sweep(keep, store=True)
    d = ch.get_draws()
    return d, crns, ch.get_state()


for B in (16, 128):
    d, _, _ = run(B, False, 700, 200)
    S = d["sqrtht_all"][:, [0, 59, 119], :, :].mean(axis=(0, 3))
    print("philox B", B, np.round(S.ravel(order="F"), 3), flush=True)
d, crns, got = run(4, True, 60, 20)
S = d["sqrtht_all"][:, [0, 59, 119], :, :].mean(axis=(0, 3))
print("crn B 4", np.round(S.ravel(order="F"), 3))
st = dict(st0)
for m in range(60):
    st = oracle.linear_sweep(st, su, crns[0][m], cta_form="syrk")
print("chain0 final sqrtht dev vs oracle", float(np.max(np.abs(got["sqrtht"][..., 0] - st["sqrtht"]))))
print("oracle final", np.round(st["sqrtht"][[0, 59, 119], :].ravel(order="F"), 3))
print("device final", np.round(got["sqrtht"][..., 0][[0, 59, 119], :].ravel(order="F"), 3))
