"""Hybrid shadow-rate model (mcmcVARhybridGibbs.m) on CPU: design and prior of the
oracle restatement against the reference's definitions, host setup == oracle
setup, the ELB conditionals in the residual form == gibbsdrawShadowrates as
written, and one oracle sweep's invariants."""
import numpy as np
import pytest

from helpers import toy_hybrid_setup


@pytest.fixture(scope="module")
def hy():
    from oracle import ccmm_oracle_hybrid
    return ccmm_oracle_hybrid


def _real(hy, oracle, fred, elb=0.25, p=12):
    ndxS, _, _ = oracle.set_shadow_yields(fred["ncode"], elb)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, elb, p)
    return hy.hybrid_setup(len(fred["ydates"]), p, 12, fred["data"], fred["ydates"], ndxS, mpm, elb, e0)


def test_hybrid_design_and_prior(hy, oracle, fred):
    """K = 1 + N p + Ns p = 277; Xffrlags = lagged actual rates floored
    at the ELB (:77-82); FFRlags prior variances (:275-291) and zero mean."""
    hs = _real(hy, oracle, fred)
    lin = hs.lin
    N, p, Ns = lin.N, lin.p, len(hs.ndxS)
    assert (lin.K, hs.Kshadow, Ns) == (277, 241, 3)
    data = lin.data
    for l in (1, 5, 12):
        for s in range(Ns):
            col = hs.Kshadow + (l - 1) * Ns + s
            want = np.maximum(data[p - l:data.shape[0] - l, hs.ndxS[s]], 0.25)
            np.testing.assert_array_equal(lin.X[:, col], want)
    assert lin.X[:, hs.Kshadow:].min() >= 0.25
    s2 = np.sum(lin.ARresid ** 2, axis=0) / (lin.T - 2)
    i, l, s = 4, 3, 1
    j = hs.ndxS[s]
    v = s2[i] / s2[j] * 0.04 * 0.25 / l ** 2
    assert abs(1.0 / lin.iVdiag[hs.Kshadow + (l - 1) * Ns + s, i] - v) < 1e-15 * v
    assert abs(1.0 / lin.iVdiag[hs.Kshadow + (l - 1) * Ns + s, j] - 0.04 / l ** 2) < 1e-17
    assert np.all(lin.iVb[hs.Kshadow:, :] == 0)
    assert hs.elbT == 165 and int(hs.sNaN.sum()) == 276


def test_host_hybrid_setup_matches_oracle(pkg, hy, oracle, fred):
    hs = _real(hy, oracle, fred)
    ndxS, _, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    hm = pkg.model.build_hybrid(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, mpm,
                                0.25, hs.elbT0)
    m = hm.var
    assert (m.K, hm.Kshadow, hm.elbT) == (hs.lin.K, hs.Kshadow, hs.elbT)
    np.testing.assert_array_equal(m.X, hs.lin.X)
    np.testing.assert_allclose(m.iVdiag, hs.lin.iVdiag, rtol=1e-14)
    np.testing.assert_array_equal(m.iVb, hs.lin.iVb)
    np.testing.assert_array_equal(m.Xjumpoff, hs.lin.Xjumpoff)
    np.testing.assert_array_equal(hm.sNaN, hs.sNaN)


@pytest.mark.parametrize("burn", [0, 3])
def test_hybrid_elb_stable_matches_qr_toy(hy, burn):
    """Hybrid state space (companion from PAI(1:Kshadow,:), Yhatactual from the
    Xffrlags block): residual form == as-written QR form."""
    from oracle import ccmm_oracle as O
    from oracle import elb_fast as F
    hs = toy_hybrid_setup(hy)
    lin = hs.lin
    rng = np.random.default_rng(11)
    st = hy.hybrid_init_state(hs)
    A = np.eye(lin.N) + np.tril(rng.uniform(-0.3, 0.3, (lin.N, lin.N)), -1)
    sqrtht = np.exp(np.cumsum(0.05 * rng.standard_normal((lin.T, lin.N)), axis=0) / 2)
    # a stable companion (the X0\\Y0 start of the toy data is explosive: its shadow-rate
    # and Xffrlags columns are nearly collinear, and the as-written form then loses all digits)
    PAI = np.zeros((lin.K, lin.N))
    PAI[0, :] = 0.1
    PAI[1 + np.arange(lin.N), np.arange(lin.N)] = 0.5
    PAI[hs.Kshadow:, :] = rng.uniform(-0.1, 0.1, (lin.K - hs.Kshadow, lin.N))
    C, Psi, SVol, Yhat = hy.elb_state_space(hs, PAI, np.linalg.inv(A), sqrtht)
    assert C.shape == (hs.Kshadow, hs.Kshadow) and np.any(Yhat != 0)
    u = hy.hybrid_draw_crn(rng, hs)["uELB"]
    elbY = st["Y"][hs.elbT0:, :].T
    a = O.gibbsdraw_shadowrates(elbY, hs.X0, Yhat, hs.ndxSmask, hs.sNaN, lin.p, C, Psi, SVol,
                                hs.ELB, 1, burn, u)
    b = F.gibbsdraw_shadowrates_stable(elbY, hs.X0, Yhat, hs.ndxSmask, hs.sNaN, lin.p, C, Psi,
                                       SVol, hs.ELB, 1, burn, u)
    assert np.max(np.abs(a - b)) < 1e-10


def test_hybrid_sweep_oracle_toy(hy):
    """One hybrid oracle sweep: censored cells respect the ELB, uncensored cells keep
    their data, the lag columns are rebuilt from the draws, Xffrlags stay fixed."""
    hs = toy_hybrid_setup(hy)
    st = hy.hybrid_init_state(hs)
    out = hy.hybrid_sweep(st, hs, hy.hybrid_draw_crn(np.random.default_rng(2), hs))
    S = out["shadowrate"]
    assert np.all(S[hs.sNaN] <= hs.ELB + 1e-12)
    Yw = hs.lin.Y[hs.elbT0:, hs.ndxS].T
    np.testing.assert_array_equal(S[~hs.sNaN], Yw[~hs.sNaN])
    np.testing.assert_array_equal(out["X"][:, hs.Kshadow:], hs.Xffrlags)
    p, N = hs.lin.p, hs.lin.N
    for l in range(1, p + 1):
        np.testing.assert_array_equal(out["X"][hs.elbT0 + l:, 1 + (l - 1) * N + hs.ndxS],
                                      out["Y"][hs.elbT0:hs.lin.T - l, hs.ndxS])
    assert out["PAI"].shape == (hs.lin.K, N)
