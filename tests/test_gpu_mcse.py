"""Monte Carlo parity of the production (Philox) path: posterior means of the linear
BVAR-SV on the toy design of tools/make_mcse_fixture.py, from 128 device chains (500 burn-in
+ 200 stored sweeps each), against one long oracle chain (2000 kept sweeps) committed as
tests/golden/mcse_toy.npz.  Numerical standard errors as Diagnostics.m:134-300 (momentg,
15 % taper); the device NSE pools the chains' (independent) NSEs.  Every one of the 64
quantities (PAI, free A entries, vech PHI, sqrtht at three months) must agree within
4.5 combined standard errors; a different generator stream makes this the test that the
draws come from the same posterior, not that they equal the oracle's."""
import numpy as np
import pytest

from conftest import ROOT
from helpers import toy_setup

pytestmark = pytest.mark.gpu


def test_posterior_means_within_mcse(pkg, ctx, oracle):
    from oracle.ccmm_oracle_stats import momentg
    g = np.load(ROOT / "tests" / "golden" / "mcse_toy.npz")
    su = toy_setup(oracle, N=4, p=2, Tobs=122, seed=11)
    N, K, T = su.N, su.K, su.T
    B, burn, keep = 128, 500, 200
    ch = pkg.Chains(ctx, N=N, p=su.p, T=T, B=B, crn=False, store_capacity=keep, seed=777)
    ch.set_data(0, su.Y, su.X, su.iVdiag, su.iVb, su.sPHI, su.Vol_0mean, su.Vol_0vcvsqrt)
    st = oracle.init_state(su)
    ch.set_state(*[np.repeat(st[k][..., None], B, axis=-1) for k in ("PAI", "A", "sqrtht", "h",
                                                                         "sqrtPHI")])
    ch.sweep(burn)
    ch.sweep(keep, store=True)
    d = ch.get_draws()
    assert not ch.get_status().any()
    tsel = list(g["tsel"])
    means, nses = [], []
    for c in range(B):
        P = d["PAI_all"][:, :, :, c].reshape(keep, K * N, order="F")
        invA = d["invA_all"][:, :, :, c]
        A = np.linalg.inv(invA)
        af = np.concatenate([A[:, i, :i] for i in range(1, N)], axis=1)
        S = d["sqrtht_all"][:, :, :, c][:, tsel, :].reshape(keep, len(tsel) * N, order="F")
        Dc = np.hstack([P, af, d["PHI_all"][:, :, c], S])
        mg = momentg(Dc)
        means.append(mg["pmean"])
        nses.append(mg["nse3"])
    m_gpu = np.mean(means, axis=0)
    # independent chains: the spread of the chain means is the device estimate's MCSE
    # (robust to autocorrelation longer than momentg's 15 % taper of 200 draws sees)
    nse_gpu = np.std(means, axis=0, ddof=1) / np.sqrt(B)
    z = (m_gpu - g["pmean"]) / np.sqrt(g["nse3"] ** 2 + nse_gpu ** 2)
    print("max |z|", np.abs(z).max(), "median |z|", np.median(np.abs(z)))
    for q in np.argsort(-np.abs(z))[:6]:
        print(f"  q{q}: gpu {m_gpu[q]:.5f} +- {nse_gpu[q]:.5f}  oracle {g['pmean'][q]:.5f} +- {g['nse3'][q]:.5f}"
              f"  (nse {g['nse'][q]:.5f} nse1 {g['nse1'][q]:.5f})  z {z[q]:.2f}")
    assert np.abs(z).max() < 4.5, np.round(z, 2)
