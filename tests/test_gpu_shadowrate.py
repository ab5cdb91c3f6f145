"""mcmcVARshadowrate.m on the device (CCMM_MODEL_SHADOWRATE): CRN parity of the sweep with
the block-hybrid oracle without an actual-rate block (CTA on the shadow-rate design for
every equation, YHAT0 = []) on a toy panel and on the real C3 data (1e-9 against the device-order
CTA mirror), and the product wrapper samplers.mcmcVARshadowrate end to end (outputs 1-17, the
censored recursion flooring ndxOTHERYIELDS only)."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import random_state, synth_bh_data

pytestmark = pytest.mark.gpu


def _toy(bh, seed=3):
    N, p, Tobs, ndxS, ndxO = 5, 2, 150, (2, 3), (4,)
    data = synth_bh_data(N, p, Tobs, ndxS=ndxS, seed=seed)
    hit = np.any(data[:, list(ndxS)] <= 0.25, axis=1)
    elbT0 = int(np.argmax(hit)) - p
    bs = bh.bh_setup(Tobs, p, 12, data, np.arange(Tobs, dtype=float), np.asarray(ndxS),
                     np.asarray(ndxO), np.ones(N), 0.25, elbT0)
    bs.actualrateBlock[:] = False                  # mcmcVARshadowrate: no actual-rate block
    return bs, data


def test_shadowrate_sweep_crn(pkg, ctx, oracle):
    from oracle import ccmm_oracle_bh as bh
    from helpers import bh_crn_flat
    bs, _ = _toy(bh)
    lin = bs.lin
    B, nsw = 3, 2
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=30 + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(30)
    crns = [[bh.bh_draw_crn(rng, bs) for _ in range(nsw)] for _ in range(B)]
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=True, model=pkg.MODEL_SHADOWRATE,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, None)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    flat = np.stack([np.stack([bh_crn_flat(bh, crns[c][m], bs) for m in range(nsw)], -1)
                     for c in range(B)], -1)
    ch.sweep(nsw, crn=flat)
    got = ch.get_state()
    S = ch.get_shadowrate()
    for c in range(B):
        st = sts[c]
        for m in range(nsw):
            st = bh.bh_sweep(st, bs, crns[c][m], elb_impl="stable")
        e = max(rel_err(got["PAI"][..., c], st["PAI"], 1e-2), rel_err(S[:, :, c], st["shadowrate"], 0.1),
                rel_err(got["sqrtht"][..., c], st["sqrtht"]))
        assert e < 1e-8, (c, e)


def test_shadowrate_sweep_crn_real(pkg, ctx, oracle, fred):
    """mcmcVARshadowrate.m on the config C3 data (fredblockMD20, ELB 0.25, p = 12; three shadow
    rates, elbT = 165): CTA on the shadow-rate design for every equation (no actual-rate block),
    two chained CRN sweeps against the oracle with CTAsys in the device's operation order
    (oracle/cta_mirror.cta, cta_form="mirror"): the north star's 1e-9 on PAI, A, sqrtht, sqrtPHI, the
    shadow rates and the rebuilt X / Y, drawTruncNormal branches and KSC indicators bit-exact."""
    from oracle import ccmm_oracle_bh as bh
    from test_gpu_bh import _check, _real_bs, _run
    bs = _real_bs(bh, oracle, fred)
    bs.actualrateBlock[:] = False                  # mcmcVARshadowrate: no actual-rate block
    out = _run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=2, seed=70, shadowrate_model=True)
    _check(oracle, bs, *out, tol_pai=1e-9, tol_s=1e-9)


def test_mcmcVARshadowrate_wrapper(pkg, fred):
    S = pkg.samplers
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    e0 = pkg.model.elbT0_of(fred["data"], ndxS, 0.25, 12)
    thisT = len(fred["ydates"]) - 24
    yreal = S.realized_values(fred["data"], thisT, 12, ndxS, 0.25)
    stats = {}
    out = S.mcmcVARshadowrate(thisT, 6, 12, 12, fred["data"], fred["ydates"], mpm, True, False, ndxS,
                              ndxO, True, 0.25, e0, yrealized=yreal, fcstNdraws=12, fcstNhorizons=12,
                              burnin=4, gibbsburn=5, nchains=2, stats=stats)
    assert len(out) == 17
    fYd, fYhat, fYc, fYcHat, fSd, fSh, RB = out[6:13]
    N = fred["data"].shape[1]
    assert fYd.shape == (N, 12, 12, 2) and RB.shape == (N, 12, 2)
    assert np.all(fYd[ndxY] >= 0.25) and np.all(fYc[ndxS] >= 0.25)
    assert np.all(np.isfinite(out[13]))                 # censored log scores
    assert np.array_equal(fSd, fSd)                     # uncensored shadow paths present
    assert "countELBaccept" in stats and out[16].shape == (6, 2)
