"""GPU parity of the coefficient block's QR fallback (CTA.m:80-92, CTAsys.m:90-100): a chain
whose posterior precision fails the device Cholesky is redrawn by the host QR branch of
Kailath's array from the same previous draw and normals (ccmm_host_cta.cpp).

CCMM_FORCE_QR=1 sends every chain through that branch, so the test compares it with the
oracle's QR branch (oracle.cta(..., force_qr=True): numpy/LAPACK QR of the kron-stacked
matrix, exactly as CTA.m:87).  Tolerance: |delta| / max(|x|, sd_post) < 1e-9.  A system
whose QR factor is itself singular returns CCMM_ERR_NOTSPD."""

import numpy as np
import pytest

from conftest import rel_err
from helpers import crn_flat, random_state, toy_setup

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_qr(ctx):
    with ctx.options(force_qr=1):  # every chain through the host QR branch (chain sets inherit it)
        yield


def test_cta_qr_branch(ctx, oracle, force_qr):
    su = toy_setup(oracle, N=4, p=2, Tobs=62)
    rng = np.random.default_rng(3)
    B = 3
    sts = [random_state(oracle, su, seed=10 + c) for c in range(B)]
    zs = [rng.standard_normal((su.K, su.N)) for _ in range(B)]
    got, status = ctx.cta(su.Y, su.X, np.stack([s["A"] for s in sts], -1),
                          np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb,
                          np.stack([s["PAI"] for s in sts], -1), np.stack(zs, -1))
    assert np.all(status == 1)  # "switching to QR routine" (CTA.m:82) for every chain
    for c in range(B):
        want, st, sd = oracle.cta(su.Y, su.X, su.N, su.K, sts[c]["A"], sts[c]["sqrtht"], su.iVdiag,
                                  su.iVb, sts[c]["PAI"], zs[c], return_sd=True, force_qr=True)
        assert st == 1
        e = rel_err(got[..., c], want, sd)
        print("qr branch chain", c, e)
        assert e < 1e-9, e


def test_ctasys_qr_branch(ctx, oracle, force_qr):
    su = toy_setup(oracle, N=5, p=3, Tobs=90, seed=2)
    rng = np.random.default_rng(9)
    XX = np.repeat(su.X[:, :, None], su.N, axis=2)
    XX[:, 1:, 3:] += 0.1 * rng.standard_normal((su.T, su.K - 1, su.N - 3))
    sts = [random_state(oracle, su, seed=8 + c) for c in range(2)]
    zs = [rng.standard_normal((su.K, su.N)) for _ in range(2)]
    got, status = ctx.cta(su.Y, XX, np.stack([s["A"] for s in sts], -1),
                          np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb,
                          np.stack([s["PAI"] for s in sts], -1), np.stack(zs, -1))
    assert np.all(status == 1)
    for c in range(2):
        want, _, sd = oracle.cta_sys(su.Y, XX, su.N, su.K, su.T, sts[c]["A"], sts[c]["sqrtht"],
                                     su.iVdiag, su.iVb, sts[c]["PAI"], zs[c], return_sd=True,
                                     force_qr=True)
        assert rel_err(got[..., c], want, sd) < 1e-9


def test_sweep_qr_branch(pkg, ctx, oracle, force_qr):
    """Two CRN sweeps of a chain set whose coefficient block always takes the QR branch:
    the redrawn PAI feeds the A / SV / PHI blocks of the same sweep (RESID recomputed)."""
    su = toy_setup(oracle, N=4, p=2, Tobs=80, seed=5)
    B, nsweeps = 2, 2
    sts = [random_state(oracle, su, seed=30 + c) for c in range(B)]
    rng = np.random.default_rng(8)
    crns = [[oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI) for _ in range(nsweeps)]
            for _ in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True)
    ch.set_data(0, su.Y, su.X, su.iVdiag, su.iVb, su.sPHI, su.Vol_0mean, su.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([crn_flat(oracle, crns[c][m], su) for m in range(nsweeps)], -1)
                     for c in range(B)], -1)
    ch.sweep(nsweeps, crn=flat)
    got = ch.get_state()
    status = ch.get_status()
    assert np.all(status == 1)
    for c in range(B):
        st = sts[c]
        for m in range(nsweeps):
            st = oracle.linear_sweep(st, su, crns[c][m], force_qr=True)
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, st["A"], st["sqrtht"], su.iVdiag, su.iVb,
                              st["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3)}
        print("chain", c, e)
        assert max(e.values()) < 1e-9, e


def test_cta_singular_qr_is_an_error(ctx, oracle):
    """A coefficient with a zero prior precision and an all-zero regressor: the Cholesky
    pivot is 0, the QR factor is singular too (MATLAB would return Inf); the call fails
    with CCMM_ERR_NOTSPD instead of returning non-finite draws silently."""
    su = toy_setup(oracle, N=3, p=2, Tobs=60, seed=1)
    X = su.X.copy()
    X[:, 2] = 0.0
    iVd = su.iVdiag.copy()
    iVd[2, :] = 0.0
    st = random_state(oracle, su, seed=4)
    with pytest.raises(RuntimeError, match="rc=-4"):
        ctx.cta(su.Y, X, st["A"][..., None], st["sqrtht"][..., None], iVd, su.iVb,
                st["PAI"][..., None], np.zeros((su.K, su.N, 1)))
