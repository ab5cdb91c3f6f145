"""Block-hybrid oracle checks on CPU: the per-month conditional formulation the
GPU kernels use (oracle/elb_fast.py) reproduces gibbsdrawShadowrates as written
(QR smoothing weights, gibbsdrawShadowrates.m:74-218), and the host setup of
mcmcVARshadowrateBlockHybrid.m matches the oracle's."""
import numpy as np
import pytest

from helpers import toy_bh_setup
from conftest import CSV


@pytest.fixture(scope="module")
def bh():
    from oracle import ccmm_oracle_bh
    return ccmm_oracle_bh


def _elb_inputs(bh, bs, seed):
    from oracle import ccmm_oracle as O
    lin = bs.lin
    rng = np.random.default_rng(seed)
    st = bh.bh_init_state(bs)
    A = np.eye(lin.N) + np.tril(rng.uniform(-0.3, 0.3, (lin.N, lin.N)), -1)
    sqrtht = np.exp(np.cumsum(0.05 * rng.standard_normal((lin.T, lin.N)), axis=0) / 2)
    C, Psi, SVol, Yhat = bh.elb_state_space(bs, st["PAI"], np.linalg.inv(A), sqrtht)
    crn = bh.bh_draw_crn(rng, bs)
    return O, st, C, Psi, SVol, Yhat, crn["uELB"]


@pytest.mark.parametrize("burn", [0, 2])
def test_elb_stable_matches_qr_toy(bh, burn):
    """The residual form the GPU evaluates (no Y0 path) == the as-written QR form."""
    from oracle import elb_fast as F
    bs = toy_bh_setup(bh)
    O, st, C, Psi, SVol, Yhat, u = _elb_inputs(bh, bs, 5)
    elbY = st["Y"][bs.elbT0:, :].T
    a = O.gibbsdraw_shadowrates(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, bs.lin.p, C, Psi, SVol,
                                bs.ELB, 1, burn, u)
    b = F.gibbsdraw_shadowrates_stable(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, bs.lin.p, C, Psi,
                                       SVol, bs.ELB, 1, burn, u)
    assert np.max(np.abs(a - b)) < 1e-10


def test_elb_stable_explosive_companion(bh, oracle, fred):
    """Explosive shadow companion matrix (spectral radius > 1, as posterior draws of
    PAIshadow can have): Y0 grows geometrically over the 165-month window and the
    as-written Ytilde = Y - Y0 loses its digits.  The stable form agrees with the
    as-written one while |Y0| is moderate and stays data-scale afterwards."""
    from oracle import elb_fast as F
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    bs = bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                     0.25, e0)
    lin = bs.lin
    st = bh.bh_init_state(bs)
    PAI = st["PAI"].copy()
    for s in bs.ndxS:
        PAI[1 + s, s] *= 1.3                        # own first lag of the shadow rates
    C, Psi, SVol, Yhat = bh.elb_state_space(bs, PAI, np.eye(lin.N), st["sqrtht"])
    rho = np.max(np.abs(np.linalg.eigvals(C)))
    assert rho > 1.2
    Y0 = F.y0_path(C, bs.X0, Yhat, lin.N, bs.elbT)
    big = np.max(np.abs(Y0), axis=0)
    u = bh.bh_draw_crn(np.random.default_rng(8), bs)["uELB"]
    elbY = st["Y"][bs.elbT0:, :].T
    a = oracle.gibbsdraw_shadowrates(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, 12, C, Psi, SVol,
                                     0.25, 1, 0, u)[:, :, 0]
    b = F.gibbsdraw_shadowrates_stable(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, 12, C, Psi, SVol,
                                       0.25, 1, 0, u)[:, :, 0]
    early = big < 1e4
    assert early.sum() > 20 and big.max() > 1e12
    assert np.max(np.abs(a - b)[:, early]) < 1e-8
    assert np.all(np.isfinite(b)) and np.max(np.abs(b)) < 50
    assert np.all(b[bs.sNaN] <= 0.25 + 1e-12)


@pytest.mark.parametrize("burn", [0, 2])
def test_elb_fast_matches_qr_toy(bh, burn):
    from oracle import elb_fast as F
    bs = toy_bh_setup(bh)
    O, st, C, Psi, SVol, Yhat, u = _elb_inputs(bh, bs, 5)
    elbY = st["Y"][bs.elbT0:, :].T
    a = O.gibbsdraw_shadowrates(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, bs.lin.p, C, Psi, SVol,
                                bs.ELB, 1, burn, u)
    b = F.gibbsdraw_shadowrates_fast(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, bs.lin.p, C, Psi,
                                     SVol, bs.ELB, 1, burn, u)
    assert np.max(np.abs(a - b)) < 1e-10
    assert np.all(a[:, :, 0][bs.sNaN] <= bs.ELB + 1e-12)


@pytest.mark.slow
def test_elb_fast_matches_qr_real(bh, oracle, fred):
    """Real data (elbT = 165, 109 censored months, 276 cells), 3 burn-in passes."""
    from oracle import elb_fast as F
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    bs = bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                     0.25, e0)
    O, st, C, Psi, SVol, Yhat, u = _elb_inputs(bh, bs, 6)
    elbY = st["Y"][bs.elbT0:, :].T
    a = O.gibbsdraw_shadowrates(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, 12, C, Psi, SVol, 0.25, 1,
                                3, u)
    b = F.gibbsdraw_shadowrates_fast(elbY, bs.X0, Yhat, bs.ndxSmask, bs.sNaN, 12, C, Psi, SVol,
                                     0.25, 1, 3, u)
    assert np.max(np.abs(a - b)) < 1e-8


def test_host_bh_setup_matches_oracle(pkg, bh, oracle, fred):
    ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    e0 = pkg.model.elbT0_of(fred["data"], ndxS, 0.25, 12)
    assert e0 == oracle.elb_t0(fred["data"], ndxS, 0.25, 12) == 585
    bm = pkg.model.build_bh(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO,
                            mpm, 0.25, e0)
    bs = bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                     0.25, e0)
    assert bm.elbT == bs.elbT == 165
    np.testing.assert_array_equal(bm.sNaN, bs.sNaN)
    np.testing.assert_array_equal(bm.actual_block, bs.actualrateBlock)
    np.testing.assert_array_equal(bm.var.X, bs.Xactual)
    assert not bm.warn_elbT0


def test_bh_sweep_oracle_toy(bh):
    """One block-hybrid oracle sweep on toy data: censored cells respect the ELB,
    uncensored cells keep their data, X/Y are rebuilt from the draws."""
    bs = toy_bh_setup(bh)
    st = bh.bh_init_state(bs)
    crn = bh.bh_draw_crn(np.random.default_rng(2), bs)
    out = bh.bh_sweep(st, bs, crn)
    S = out["shadowrate"]
    assert np.all(S[bs.sNaN] <= bs.ELB + 1e-12)
    Yw = bs.lin.Y[bs.elbT0:, bs.ndxS].T
    np.testing.assert_array_equal(S[~bs.sNaN], Yw[~bs.sNaN])
    np.testing.assert_array_equal(out["Y"][bs.elbT0:, bs.ndxS], S.T)
    p, N = bs.lin.p, bs.lin.N
    for l in range(1, p + 1):  # X lag columns hold the shadow rates
        np.testing.assert_array_equal(out["X"][bs.elbT0 + l:, 1 + (l - 1) * N + bs.ndxS],
                                      out["Y"][bs.elbT0:bs.lin.T - l, bs.ndxS])


def test_ps_joint_matches_gibbs_conditionals(bh):
    """The PS proposal density (precision_sampler_nan: joint Gaussian of all censored cells
    from the stacked VAR likelihood) and the Gibbs sampler's per-month conditionals
    (elb_fast, what k_elb_cond evaluates) share the precision: the conditional covariance
    of month t's censored cells given the other censored cells agrees.  The means differ by
    the reference's own model difference: gibbsdrawShadowrates.m:157-165 treats YHAT0 as a
    measurement offset of a VAR on Y - Y0 (and lags Y0 one period), while the PS call
    enters Yhatactual as an intercept (pai0, mcmcVARshadowrateBlockHybrid.m:423); the
    device evaluates each branch's own mean (k_elb_cond: Gibbs a_t, PS b_t)."""
    from oracle import elb_fast as F
    bs = toy_bh_setup(bh)
    O, st, C, Psi, SVol, Yhat, _ = _elb_inputs(bh, bs, 11)
    rng = np.random.default_rng(11)
    lin = bs.lin
    A = np.linalg.inv(Psi[1:1 + lin.N, :])
    sqrtht = np.ones((lin.T, lin.N))
    sqrtht[bs.elbT0:, :] = SVol.T
    args = bh.ps_inputs(bs, st["PAI"], A, sqrtht)
    n = int(bs.sNaN.sum())
    Z = np.concatenate([np.zeros((n, 1)), np.eye(n)], axis=1)
    YY = bh.precision_sampler_nan(*args, Z)
    m = args[3].ravel(order="F")
    X = YY[m, :]
    mu = X[:, 0]
    Lt = X[:, 1:] - mu[:, None]                 # L'^-1
    Sig = Lt @ Lt.T
    Prec = np.linalg.inv(Sig)
    # cell index of (series si, month t) in the missing vector (month-major)
    idx = -np.ones(bs.sNaN.shape, int)
    idx.T[bs.sNaN.T] = np.arange(n)
    elbY = st["Y"][bs.elbT0:, :].T
    Yb = elbY.copy()
    S = np.flatnonzero(bs.ndxSmask)
    tmp = Yb[S, :]
    tmp[bs.sNaN] = 0.0
    Yb[S, :] = tmp
    e0 = F.e0_path(C, bs.X0, Yhat, lin.N, bs.elbT, lin.p)
    cond = F.elb_conditionals_stable(Yb, e0, bs.ndxSmask, bs.sNaN, lin.p, C, Psi, SVol)
    worst = 0.0
    for t, (base, coef, Om) in cond.items():
        c = np.flatnonzero(bs.sNaN[:, t])
        o = np.flatnonzero(~bs.sNaN[:, t])
        ci = idx[c, t]
        # joint: covariance of x_c given the other censored cells
        jc = np.linalg.inv(Prec[np.ix_(ci, ci)])
        # Gibbs record: all Ns cells of month t given the neighbours, then given the observed
        gc = Om[np.ix_(c, c)]
        if o.size:
            gc = gc - Om[np.ix_(c, o)] @ np.linalg.solve(Om[np.ix_(o, o)], Om[np.ix_(o, c)])
        worst = max(worst, np.max(np.abs(jc - gc)) / np.max(np.abs(gc)))
    assert worst < 1e-9, worst
    # and the draws: proposal k = mu + L'^-1 z_k
    z = rng.standard_normal((n, 3))
    YY3 = bh.precision_sampler_nan(*args, z)
    assert np.allclose(YY3[m, :], mu[:, None] + Lt @ z, atol=1e-10)
    assert np.array_equal(YY3[~m, :], np.repeat(args[2].ravel(order="F")[~m][:, None], 3, 1))
