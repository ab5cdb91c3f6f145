"""GPU parity of the large-N Gibbs blocks (ccmm_bign.hip; 32 < N <= 128, the S120
configuration N = 120) and of full sweeps that run every block on the large path
(ccmm_big.hip CTA, k_astep_big, k_sv_big, k_phi_big, the N > 64 ELB kernels) against the
oracle on common random numbers.

SV convention for N > 32: the time-ordered block Cholesky sampler
(oracle.sv_draw_sequential; oracle.sv_ksc_corrsqrt switches to it above N = 32, as the
GPU does).  KSC indicators: bit-exact.  Tolerances as tests/test_gpu_parity.py: blocks
1e-9 relative (A: in units of max(|x|, sd_post)), sweeps in units of max(|x|, sd_post)."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import bh_crn_flat, crn_flat, random_state, toy_bh_setup, toy_setup

pytestmark = pytest.mark.gpu


def _resid(rng, st):
    """Residuals RESID = (A^{-1} diag(sqrtht_t) e_t)' of full column rank (OLS residuals of
    the toy VAR would have rank T - K < N at these sizes)."""
    T, N = st["sqrtht"].shape
    e = rng.standard_normal((T, N)) * st["sqrtht"]
    return np.linalg.solve(st["A"], e.T).T


@pytest.mark.parametrize("N,T", [(40, 100), (120, 160)])
def test_bign_astep(ctx, oracle, N, T):
    su = toy_setup(oracle, N=N, p=1, Tobs=T + 1, seed=4)
    st = random_state(oracle, su, seed=2)
    rng = np.random.default_rng(1)
    RESID = _resid(rng, st)
    B = 2
    zs = [rng.standard_normal(N * (N - 1) // 2) for _ in range(B)]
    shs = [st["sqrtht"] * np.exp(0.1 * c) for c in range(B)]
    gA, ginvA = ctx.astep(np.stack([RESID] * B, -1), np.stack(shs, -1), np.stack(zs, -1))
    for c in range(B):
        A, invA = oracle.a_step(RESID, shs[c], zs[c])
        # in units of the posterior sd of A: at N = 120, T = 160 the 119-regressor Gram has
        # cond ~1e5 and the summation order alone moves A by ~2e-10 relative
        eA = rel_err(gA[..., c], A, oracle.a_step_sd(RESID, shs[c]))
        ei = rel_err(ginvA[..., c], invA, 1e-3)
        print("astep N", N, "chain", c, eA, ei)
        assert eA < 1e-9 and ei < 1e-9


@pytest.mark.parametrize("N,T", [(40, 120), (120, 60)])
def test_bign_sv_sequential(ctx, oracle, N, T):
    su = toy_setup(oracle, N=N, p=1, Tobs=T + 1, seed=6)
    st = random_state(oracle, su, seed=3)
    rng = np.random.default_rng(2)
    RESID = _resid(rng, st)
    logy2 = np.log((RESID @ st["A"].T) ** 2 + su.logy2offset)
    u = rng.random((su.N, su.T))
    z = rng.standard_normal((su.N, su.T + 1))
    h, h0, sh, kai = oracle.sv_ksc_corrsqrt(logy2.T, st["h"].T, st["sqrtPHI"], su.Vol_0mean,
                                           su.Vol_0vcvsqrt, u, z)
    gh, gh0, gsh, gkai = ctx.sv_ksc(logy2.T[..., None], st["h"].T[..., None],
                                    st["sqrtPHI"][..., None], su.Vol_0mean, su.Vol_0vcvsqrt,
                                    u[..., None], z[..., None])
    np.testing.assert_array_equal(gkai[..., 0], kai)
    e = (rel_err(gh[..., 0], h, 1.0), rel_err(gsh[..., 0], sh, 1e-2), rel_err(gh0[:, 0], h0, 1.0))
    print("sv N", N, e)
    assert max(e) < 1e-9, e


@pytest.mark.parametrize("N,T", [(40, 120), (120, 200)])
def test_bign_phi_iw(ctx, oracle, N, T):
    su = toy_setup(oracle, N=N, p=1, Tobs=T + 1, seed=6)
    rng = np.random.default_rng(11)
    eta = 0.1 * rng.standard_normal((su.T, su.N))
    Z = rng.standard_normal((su.N, su.T + su.dPHI))
    sq, PHI = oracle.phi_iw(eta, su.sPHI, Z)
    gsq, gPHI = ctx.phi_iw(eta[..., None], su.sPHI, su.dPHI, Z[..., None])
    e = (rel_err(gPHI[..., 0], PHI, np.abs(PHI).max()), rel_err(gsq[..., 0], sq, np.abs(sq).max()))
    print("phi N", N, e)
    assert max(e) < 1e-11, e


def test_bign_linear_sweep_crn(pkg, ctx, oracle):
    """Two chained linear sweeps, N = 40, p = 2 (K = 81), T = 148, three chains."""
    su = toy_setup(oracle, N=40, p=2, Tobs=150, seed=8)
    B, nsweeps = 3, 2
    sts = [random_state(oracle, su, seed=100 + c) for c in range(B)]
    rng = np.random.default_rng(21)
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
    assert not ch.get_status().any()
    for c in range(B):
        st = sts[c]
        for m in range(nsweeps):
            prev = st["sqrtht"]
            st = oracle.linear_sweep(st, su, crns[c][m])
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, st["A"], st["sqrtht"], su.iVdiag, su.iVb,
                              st["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], prev)),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3)}
        print("chain", c, e)
        assert max(e.values()) < 1e-10, e


@pytest.mark.parametrize("N", [40, 72])
def test_bign_bh_sweep_crn(pkg, ctx, oracle, N):
    """Block-hybrid sweep on the large path: N = 40 and N = 72 (the ELB kernels' lanes own
    two equations), p = 2, T = 298, two shadow rates with mixed censoring, one other yield."""
    from oracle import ccmm_oracle_bh as bh
    bs = toy_bh_setup(bh, N=N, Tobs=300, ndxS=(N - 4, N - 3), ndxO=(N - 2,))
    lin = bs.lin
    B, nsweeps = 2, 1
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=50 + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(7)
    crns = [[bh.bh_draw_crn(rng, bs) for _ in range(nsweeps)] for _ in range(B)]
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=True, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([bh_crn_flat(bh, crns[c][m], bs) for m in range(nsweeps)], -1)
                     for c in range(B)], -1)
    ch.sweep(nsweeps, crn=flat)
    got = ch.get_state()
    S = ch.get_shadowrate()
    assert not ch.get_status().any()
    for c in range(B):
        st = sts[c]
        for m in range(nsweeps):
            prev = st["sqrtht"]
            st = bh.bh_sweep(st, bs, crns[c][m], elb_impl="stable")
        XX = np.empty((lin.T, lin.K, lin.N))
        XX[:, :, bs.actualrateBlock] = bs.Xactual[:, :, None]
        XX[:, :, ~bs.actualrateBlock] = st["X"][:, :, None]
        _, _, sd = oracle.cta_sys(st["Y"], XX, lin.N, lin.K, lin.T, st["A"], st["sqrtht"],
                                  lin.iVdiag, lin.iVb, st["PAI"], np.zeros((lin.K, lin.N)),
                                  return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], prev)),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3),
             "shadowrate": rel_err(S[:, :, c], st["shadowrate"], 0.1)}
        print("N", N, "chain", c, e)
        assert max(e.values()) < 1e-10, e
        assert np.all(S[:, :, c][bs.sNaN] <= bs.ELB + 1e-12)
