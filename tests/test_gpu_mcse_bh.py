"""Monte Carlo parity of the block-hybrid production path with the acceptance-sampling ELB
branch (Philox): posterior means on the toy panel of tools/make_mcse_bh_fixture.py from 128
device chains (300 burn-in + 200 stored sweeps each, 1000 PS proposals with Gibbs fallback at
every sweep) against one long oracle chain (2000 kept sweeps of bh_sweep(use_ps=True))
committed as tests/golden/mcse_bh_toy.npz.  Quantities: PAI, the free A entries, vech PHI,
sqrtht at three months and every censored shadow rate; each within 4.5 combined standard
errors (MCSE as in test_gpu_mcse.py)."""
import importlib.util

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bh_ps_posterior_means_within_mcse(pkg, ctx, oracle):
    from oracle import ccmm_oracle_bh as bh
    g = np.load(ROOT / "tests" / "golden" / "mcse_bh_toy.npz")
    spec = importlib.util.spec_from_file_location("tps", ROOT / "tests" / "test_gpu_ps.py")
    t = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(t)
    bs = t._toy_bs(bh, (114, 120), valley=True)
    lin = bs.lin
    N, K, T = lin.N, lin.K, lin.T
    B, burn, keep = 128, 300, 200
    ch = pkg.Chains(ctx, N=N, p=lin.p, T=T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                    store_capacity=keep, seed=4242)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_elb_ps(int(g["nproposals"]), 1)
    st = bh.bh_init_state(bs)
    ch.set_state(*[np.repeat(st[k][..., None], B, axis=-1) for k in ("PAI", "A", "sqrtht", "h",
                                                                         "sqrtPHI")])
    ch.sweep(burn)
    ch.sweep(keep, store=True)
    ps = ch.get_ps()
    d = ch.get_draws()
    assert not ch.get_status().any()
    from oracle.ccmm_oracle_stats import momentg
    tsel = list(g["tsel"])
    cells = bs.sNaN.ravel(order="F")
    means = []
    for c in range(B):
        P = d["PAI_all"][:, :, :, c].reshape(keep, K * N, order="F")
        A = np.linalg.inv(d["invA_all"][:, :, :, c])
        af = np.concatenate([A[:, i, :i] for i in range(1, N)], axis=1)
        S = d["sqrtht_all"][:, :, :, c][:, tsel, :].reshape(keep, len(tsel) * N, order="F")
        R = d["shadowrate_all"][:, :, :bs.elbT, c].reshape(keep, -1, order="F")[:, cells]
        means.append(momentg(np.hstack([P, af, d["PHI_all"][:, :, c], S, R]))["pmean"])
    m_gpu = np.mean(means, axis=0)
    nse_gpu = np.std(means, axis=0, ddof=1) / np.sqrt(B)
    z = (m_gpu - g["pmean"]) / np.sqrt(g["nse3"] ** 2 + nse_gpu ** 2)
    rate = (ps["countAccept"].sum() + ps["countAcceptBurnin"].sum()) / (B * (burn + keep))
    print("accept rate", rate, "max |z|", np.abs(z).max(), "median |z|", np.median(np.abs(z)))
    assert rate > 0.1                       # the PS branch actually serves most sweeps
    assert np.abs(z).max() < 4.5, np.round(z, 2)
