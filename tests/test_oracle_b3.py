"""KATs of the gibbsdrawShadowratesB3 restatement (oracle.gibbsdraw_shadowrates_b3,
gibbsdrawShadowratesB3.m:1-231): with one censored month, the QR-built smoothing weights must give
the Gaussian conditional of the shadow rates implied directly by the VAR likelihood
    Y_tau = c + sum_l Phi_l Y_{tau-l} + B_tau diag(SVol_tau) e_tau,   e_tau ~ N(0, I)
(terms tau = t .. min(t + p, T)), with a month-varying impact matrix B_tau; the draw is then
drawTruncNormal of that conditional (sequentially over the censored series, :196-201)."""
import numpy as np
import pytest


def _var(rng, Ny, p, T):
    K = Ny * p + 1
    PAI = np.zeros((K, Ny))
    PAI[0] = rng.uniform(-0.2, 0.2, Ny)
    for l in range(p):
        PAI[1 + l * Ny:1 + (l + 1) * Ny] = (0.5 / (l + 1)) * np.eye(Ny) + 0.05 * rng.standard_normal((Ny, Ny))
    A = np.zeros((K, K))
    A[0, 0] = 1.0
    A[1:1 + Ny, :] = PAI.T
    A[1 + Ny:, 1:1 + Ny * (p - 1)] = np.eye(Ny * (p - 1))
    B = np.zeros((K, Ny, T))
    for t in range(T):
        B[1:1 + Ny, :, t] = np.eye(Ny) + np.tril(0.3 * rng.standard_normal((Ny, Ny)), -1)
    return PAI, A, B


def _brute_conditional(Y, STATE0, PAI, B, SVol, p, t0, sidx):
    """Mean and covariance of Y[sidx, t0] given everything else, from the VAR likelihood."""
    Ny, T = Y.shape
    c, Phi = PAI[0], [PAI[1 + l * Ny:1 + (l + 1) * Ny].T for l in range(p)]
    lag0 = STATE0[1:].reshape(p, Ny)  # lag l+1 block = Y_{-l}
    def ylag(Yc, tau, l):  # Y_{tau - l}
        return Yc[:, tau - l] if tau - l >= 0 else lag0[l - tau - 1]
    def resid(Yc, tau):
        r = Yc[:, tau] - c
        for l in range(1, p + 1):
            r = r - Phi[l - 1] @ ylag(Yc, tau, l)
        return np.linalg.solve(B[1:1 + Ny, :, tau], r) / SVol[:, tau]
    ns = len(sidx)
    a = []
    bcols = []
    Yz = Y.copy()
    Yz[sidx, t0] = 0.0
    for tau in range(t0, min(t0 + p, T - 1) + 1):
        a.append(resid(Yz, tau))
        cols = []
        for j in range(ns):
            Yj = Yz.copy()
            Yj[sidx[j], t0] = 1.0
            cols.append(resid(Yj, tau) - a[-1])
        bcols.append(np.stack(cols, axis=1))
    a = np.concatenate(a)
    Bm = np.vstack(bcols)
    P = Bm.T @ Bm
    m = -np.linalg.solve(P, Bm.T @ a)
    return m, np.linalg.inv(P)


@pytest.mark.parametrize("Ns", [1, 2])
def test_b3_single_month_conditional(oracle, Ns):
    rng = np.random.default_rng(7 + Ns)
    Ny, p, T, t0 = 4, 2, 14, 6
    PAI, A, B = _var(rng, Ny, p, T)
    ndxS = np.zeros(Ny, bool)
    ndxS[:Ns] = True
    sNaN = np.zeros((Ns, T), bool)
    sNaN[:, t0] = True
    Y = rng.normal(size=(Ny, T))
    Y[:Ns, t0] = 0.1
    STATE0 = np.concatenate([[1.0], rng.normal(size=Ny * p)])
    SVol = np.exp(0.2 * rng.normal(size=(Ny, T)))
    u = rng.random((Ns, T, 1))
    got, fl = oracle.gibbsdraw_shadowrates_b3(Y, STATE0, ndxS, sNaN, p, A, B, SVol, 0.25, 1, 0, u,
                                              return_flags=True)
    m, V = _brute_conditional(Y, STATE0, PAI, B, SVol, p, t0, list(range(Ns)))
    S = Y[:Ns, t0].copy()
    for s in range(Ns):  # sequential conditional draws within the month (:196-201)
        o = np.arange(Ns) != s
        if Ns == 1:
            mu, sig = m[0], np.sqrt(V[0, 0])
        else:
            beta = np.linalg.solve(V[np.ix_(o, o)], V[o, s])
            mu = m[s] + beta @ (S[o] - m[o])
            sig = np.sqrt(V[s, s] - V[s, o] @ beta)
        S[s], f = oracle.draw_trunc_normal(mu, sig, 0.25, u[s, t0, 0])
        assert fl[s, t0, 0] == f
    np.testing.assert_allclose(got[:, t0, 0], S, rtol=0, atol=1e-10)
    assert np.all(got[:, t0, 0] <= 0.25)
