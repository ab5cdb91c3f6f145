"""CPU checks of the predictive-density oracle (oracle/ccmm_oracle_fcst.py):
mvncdf restatement against scipy's Genz integrator, the censored log score's
reduction identities, and the simulation's structural properties."""
import numpy as np
import pytest
from scipy import stats

from fcst_cases import fcst_inputs


@pytest.fixture(scope="module")
def F():
    from oracle import ccmm_oracle_fcst
    return ccmm_oracle_fcst


@pytest.mark.parametrize("r", [-0.95, -0.5, 0.0, 0.2, 0.6, 0.9, 0.97])
def test_bvn_cdf_vs_scipy(F, r):
    S = np.array([[1.0, r], [r, 1.0]])
    for h, k in [(-1.0, 0.5), (0.3, 0.3), (1.5, -2.0), (-2.5, -2.2)]:
        want = stats.multivariate_normal(mean=[0, 0], cov=S).cdf([h, k])
        assert abs(F.bvn_cdf(h, k, r) - want) < 1e-7


def test_tvn_cdf_vs_scipy(F):
    rng = np.random.default_rng(0)
    for _ in range(4):
        L = np.tril(rng.uniform(-0.8, 0.8, (3, 3))) + np.diag([1.0, 0.6, 0.4])
        S = L @ L.T
        b = rng.uniform(-1, 1, 3)
        mu = rng.uniform(-0.3, 0.3, 3)
        want = stats.multivariate_normal(mean=mu, cov=S).cdf(b)
        assert abs(F.mvncdf(b, mu, S) - want) < 2e-5  # scipy is a randomized QMC rule (~1e-5)


@pytest.mark.parametrize("d", [4, 5, 6, 8])
def test_mvn_lattice_vs_scipy(F, d):
    """The declared 4+-dimensional mvncdf rule (deterministic rank-1 lattice, the device's) against
    scipy's randomised Genz lattice at tight tolerance: within 1e-6 absolute (MATLAB mvncdf's own
    tolerance at d >= 4 is 1e-4)."""
    rng = np.random.default_rng(3 + d)
    A = rng.normal(size=(d, d))
    S = A @ A.T / d + 0.3 * np.eye(d)
    b = rng.normal(size=d) * 0.8 - 0.3
    mu = rng.uniform(-0.2, 0.2, d)
    want = stats.multivariate_normal.cdf(b, mean=mu, cov=S, abseps=1e-10, releps=1e-10, maxpts=2_000_000)
    got = F.mvncdf(b, mu, S)
    print(d, got, want)
    assert abs(got - want) < 1e-6


def test_censored_one_at_elb_is_conditional_normal(F):
    """One censored series: llf = log N(y_off) + log Phi((y_at - E[y_at|y_off]) / sd)."""
    rng = np.random.default_rng(1)
    n = 4
    S = np.tril(rng.uniform(-0.5, 0.5, (n, n))) + np.eye(n)
    mu = rng.standard_normal(n)
    y = mu + rng.standard_normal(n)
    y[2] = -1.0
    Om = S @ S.T
    off = [0, 1, 3]
    c = Om[2, off] @ np.linalg.solve(Om[np.ix_(off, off)], y[off] - mu[off]) + mu[2]
    v = Om[2, 2] - Om[2, off] @ np.linalg.solve(Om[np.ix_(off, off)], Om[off, 2])
    want = stats.multivariate_normal(mu[off], Om[np.ix_(off, off)]).logpdf(y[off]) + \
        stats.norm.logcdf(y[2], c, np.sqrt(v))  # upper limit = yAtELB (:75)
    got = F.logscore_gaussian_censored(mu, S, y, -0.5, np.array([False, False, True, False]))
    assert abs(got - want) < 1e-10


def test_fcst_structure(F, oracle, fred):
    d = fcst_inputs(oracle, fred, B=1, H=12, Nd=3)
    fY, fYc, yhat, sc = F.fcst_draw(d["PAI"][..., 0], d["invA"][..., 0], d["logSV0"][:, 0],
                                    d["sqrtPHI"][..., 0], d["Xj"][:, 0], d["ys"][1], d["yields"],
                                    d["elb"], d["svz"][..., 0], d["z"][..., 0])
    assert np.all(fYc[d["yields"]] >= d["elb"])
    # before any censoring binds, the censored path equals the linear path
    first = np.argmax(np.any(fY[d["yields"]] < d["elb"], axis=0), axis=0)
    assert np.allclose(fY[:, 0, :][:, first > 0], fYc[:, 0, :][:, first > 0])
    # the X / I split of the uncensored score: the sum is the joint score when the blocks are
    # uncorrelated only, so check finiteness and the ELB <= uncensored ordering is not assumed
    assert np.all(np.isfinite(sc))
    assert np.allclose(yhat[:, 0], d["PAI"][..., 0].T @ d["Xj"][:, 0])


def test_bh_forecast_reduces_to_linear(F, oracle, fred):
    """With no actual-rate block the block-hybrid companion (K + Nyields p states) is the
    linear one: paths equal fcst_draw's, scores equal its ELB / X / I scores."""
    d = fcst_inputs(oracle, fred, B=1, H=6, Nd=3)
    N, p = 20, 12
    y = d["ys"][2]
    args = (d["PAI"][..., 0], d["invA"][..., 0], d["logSV0"][:, 0], d["sqrtPHI"][..., 0])
    fY, fYc, yhat, sc = F.fcst_draw(*args, d["Xj"][:, 0], y, d["yields"], 0.25,
                                    d["svz"][..., 0], d["z"][..., 0])
    ny = int(d["yields"].sum())
    Xj = np.concatenate([d["Xj"][:, 0], np.full(ny * p, 0.123)])  # actual lags: unused here
    bY, bsc = F.fcst_draw_bh(*args, Xj, y, d["yields"], np.zeros(N, bool), 0.25,
                             d["svz"][..., 0], d["z"][..., 0])
    np.testing.assert_allclose(bY, fY, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(bsc, sc[1:], rtol=1e-12, atol=1e-12)


def test_bh_forecast_actual_rates(F, oracle, fred):
    """The actual-rate equations read the ELB-floored yields (fcstX0(ndxfcstActual) =
    max(shadow, ELB), mcmcVARshadowrateBlockHybrid.m:623); an independent lag-ring
    restatement of the same recursion agrees with the dense-companion oracle."""
    d = fcst_inputs(oracle, fred, B=1, H=8, Nd=2)
    N, p, elb = 20, 12, 0.25
    K = N * p + 1
    yields = d["yields"]
    actual = ~yields
    PAI, invA = d["PAI"][..., 0].copy(), d["invA"][..., 0]
    PAI[0, yields] -= 0.6                          # push the yields below the ELB
    rng = np.random.default_rng(3)
    ny = np.flatnonzero(yields)
    act_lags = rng.uniform(0.0, 0.3, (p, ny.size))
    Xj = np.concatenate([d["Xj"][:, 0], act_lags.ravel()])
    y = d["ys"][0]
    fY, sc = F.fcst_draw_bh(PAI, invA, d["logSV0"][:, 0], d["sqrtPHI"][..., 0], Xj, y, yields,
                            actual, elb, d["svz"][..., 0], d["z"][..., 0])
    assert (fY[yields] < elb).any()                # the floor binds somewhere
    H, Nd = 8, 2
    svs = (d["sqrtPHI"][..., 0] @ d["svz"][..., 0]).reshape(N, H, Nd, order="F")
    for nn in range(Nd):
        sv = np.exp(0.5 * (d["logSV0"][:, 0][:, None] + np.cumsum(svs[:, :, nn], axis=1)))
        nu = invA @ (sv * d["z"][..., 0][:, :, nn])
        shadow = [Xj[1 + l * N:1 + (l + 1) * N].copy() for l in range(p)]
        mixed = [s.copy() for s in shadow]
        for l in range(p):
            mixed[l][ny] = act_lags[l]
        for hh in range(H):
            xs = np.concatenate([[1.0]] + shadow)
            xm = np.concatenate([[1.0]] + mixed)
            yv = np.where(actual, PAI.T @ xm, PAI.T @ xs) + nu[:, hh]
            np.testing.assert_allclose(fY[:, hh, nn], yv, rtol=1e-11, atol=1e-11)
            shadow = [yv.copy()] + shadow[:-1]
            ym = yv.copy()
            ym[yields] = np.maximum(ym[yields], elb)
            mixed = [ym] + mixed[:-1]
    assert np.all(np.isfinite(sc))
