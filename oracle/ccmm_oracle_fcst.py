"""Oracle (CPU restatement) of the predictive-density block of the Gibbs sweep —
TEST INFRASTRUCTURE ONLY (see ccmm_oracle.py).

Follows mcmcVAR.m:298-381 (identical in mcmcVARshadowrateBlockHybrid.m:550-669
for the linear/censored simulation) for ONE kept draw: SV shock paths, the
linear companion simulation (ltitr), the one-step predictive log scores
(logscoreGaussian.m:15-20, logscoreGaussianCensored.m:13-88), the censored
simulation (:354-372) and the Rao-Blackwellised mean path (:375-379).

PARITY UNPINNED (MATLAB reference, no fixtures).  MATLAB built-ins restated:
``normcdf`` exactly (erfc); ``mvncdf`` for 2 and 3 censored series by
independent adaptive quadrature (scipy.integrate.quad) of the conditional
univariate / bivariate integrals — MATLAB's own trivariate
tolerance is 1e-8 absolute.  With 4+ censored series MATLAB switches to a
randomised quasi-Monte Carlo rule (absolute tolerance 1e-4) that cannot be matched draw for
draw; the declared convention is a deterministic rank-1 lattice rule inside that tolerance
(``mvn_lattice_cdf``, the device's rule), itself checked against scipy's randomised Genz
lattice at 1e-6 (tests/test_oracle_fcst.py).
"""
from __future__ import annotations

import math

import numpy as np
from scipy import integrate
from scipy.special import ndtr

LOG2PI = math.log(2.0 * math.pi)


def bvn_cdf(h, k, r):
    """P(Z1 <= h, Z2 <= k) for standard normals with correlation r: the conditional
    integral  int_{-inf}^{h} phi(x) Phi((k - r x) / sqrt(1 - r^2)) dx, adaptive
    (positive by construction, also deep in the tails)."""
    if r == 0.0:
        return ndtr(h) * ndtr(k)
    s = math.sqrt(1.0 - r * r)
    f = lambda x: math.exp(-0.5 * x * x) / math.sqrt(2 * math.pi) * ndtr((k - r * x) / s)
    pts = [k / r] if -50 < k / r < h else None
    lo = min(-40.0, h - 40.0)
    val, _ = integrate.quad(f, lo, h, epsabs=1e-300, epsrel=1e-12, limit=400, points=pts)
    return val


MVN_PTS = 64 * 1024
MVN_ALPHA = np.sqrt(np.array([2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31], float))


def mvn_lattice_cdf(x, L, npts=MVN_PTS):
    """P(X <= x), X ~ N(0, L L') (L lower, d = 4..12): Genz's separation of variables on the
    rank-1 lattice w_q = |2 frac((q + 1) sqrt(prime_i)) - 1|, q = 0..npts-1 (the device's rule,
    csrc/ccmm_fcst.hip mvn_lattice_cdf; MATLAB mvncdf uses a randomised QMC rule at d >= 4)."""
    from scipy.special import ndtri
    x = np.asarray(x, float)
    d = len(x)
    e1 = ndtr(x[0] / L[0, 0])
    if not e1 > 0.0:
        return 0.0
    q = np.arange(1, npts + 1, dtype=float)
    e = np.full(npts, e1)
    f = e.copy()
    Y = np.zeros((d, npts))
    for i in range(1, d):
        w = q * MVN_ALPHA[i - 1]
        w = np.abs(2.0 * (w - np.floor(w)) - 1.0)
        Y[i - 1] = ndtri(np.clip(w * e, 1e-300, 1.0 - 1e-16))
        e = ndtr((x[i] - L[i, :i] @ Y[:i]) / L[i, i])
        f = f * e
    return float(min(1.0, max(0.0, f.mean())))


def mvncdf(b, mu, S):
    """mvncdf(b', mu', S) (MATLAB mvncdf semantics, upper limits): dimension 1..3 by adaptive
    quadrature, 4..12 by the declared lattice rule (mvn_lattice_cdf)."""
    d = len(b)
    x = (np.asarray(b, float) - np.asarray(mu, float))
    if d == 1:
        return ndtr(x[0] / math.sqrt(S[0, 0]))
    if d == 2:
        s1, s2 = math.sqrt(S[0, 0]), math.sqrt(S[1, 1])
        return bvn_cdf(x[0] / s1, x[1] / s2, S[0, 1] / (s1 * s2))
    if d == 3:
        L = np.linalg.cholesky(S)
        v2 = L[2, 1] ** 2 + L[2, 2] ** 2
        s3 = math.sqrt(v2)
        rho = L[2, 1] / s3

        def inner(z1):
            h = (x[1] - L[1, 0] * z1) / L[1, 1]
            k = (x[2] - L[2, 0] * z1) / s3
            return math.exp(-0.5 * z1 * z1) / math.sqrt(2 * math.pi) * bvn_cdf(h, k, rho)

        pts = [v for v in (x[1] / L[1, 0] if L[1, 0] else None, x[2] / L[2, 0] if L[2, 0] else None)
               if v is not None and -40 < v < x[0] / L[0, 0]]
        val, _ = integrate.quad(inner, -40.0, x[0] / L[0, 0], epsabs=1e-300, epsrel=1e-11,
                                limit=400, points=pts or None)
        return val
    if d <= 12:
        return mvn_lattice_cdf(x, np.linalg.cholesky(S))
    return float("nan")


def logscore_gaussian(mu, sqrtOmega, y, logdet=None):
    """logscoreGaussian.m:15-20 (sqrtOmega lower triangular -> triangular solve)."""
    if logdet is None:
        logdet = 2 * np.sum(np.log(np.diag(sqrtOmega)))
    from scipy.linalg import solve_triangular
    ydev = solve_triangular(sqrtOmega, y - mu, lower=True)
    return -0.5 * (len(y) * LOG2PI + logdet + np.sum(ydev ** 2))


def logscore_gaussian_censored(mu, sqrtOmega, y, elb, censorable=None):
    """logscoreGaussianCensored.m:13-88 as written (incl. the NoffELB > 1 test at :58)."""
    N = len(y)
    if censorable is None:
        censorable = np.ones(N, bool)
    at = (y <= elb) & censorable
    Nat = int(at.sum())
    Noff = N - Nat
    if Nat == 0:
        raise ValueError("logscoreGaussianCensored.m:33 references undefined muY at NatELB == 0")
    order = np.concatenate([np.nonzero(~at)[0], np.nonzero(at)[0]])
    ydev = (y - mu)[order]
    yAt, muAt = y[at], mu[at]
    S = sqrtOmega[order, :]
    L = np.linalg.cholesky(S @ S.T)
    from scipy.linalg import solve_triangular
    if Noff > 1:
        L11 = L[:Noff, :Noff]
        z1 = solve_triangular(L11, ydev[:Noff], lower=True)
        llf1 = -0.5 * (Noff * LOG2PI + 2 * np.sum(np.log(np.diag(L11))) + np.sum(z1 ** 2))
        y21 = muAt + L[Noff:, :Noff] @ z1
    else:
        llf1 = 0.0
        y21 = muAt
    L22 = L[Noff:, Noff:]
    # MATLAB's log: log(0) = -Inf (a probability that underflows)
    mlog = lambda v: math.log(v) if v > 0.0 else -math.inf
    if Nat == 1:
        llf2 = mlog(ndtr((yAt[0] - y21[0]) / L22[0, 0]))
    else:
        llf2 = mlog(mvncdf(yAt, y21, L22 @ L22.T))
    return llf1 + llf2


def fcst_draw(PAI, invA, logSV0, sqrtPHI, Xjumpoff, yrealized, ndxYields, elb, svz, z):
    """One kept draw of mcmcVAR.m:298-381.

    PAI K x N, invA N x N, logSV0 N (Vol_states(end,:)'), sqrtPHI N x N,
    Xjumpoff K, yrealized N (first column), ndxYields bool N, elb scalar,
    svz = randn(N, H*Nd) (:302), z = randn(N, H, Nd) (:306).
    Returns fcstY N x H x Nd, fcstYcensor N x H x Nd, yhat N x H,
    scores 4 x Nd (fcstLogscore, fcstLogscoreELB, fcstLogscoreX, fcstLogscoreI).
    """
    K, N = PAI.shape
    H, Nd = z.shape[1], z.shape[2]
    ndxYx = ~ndxYields
    ndxYi = ndxYields
    yNatELB = int(np.sum(yrealized[ndxYi] <= elb))
    svshocks = (sqrtPHI @ svz).reshape(N, H, Nd, order="F")
    fY = np.empty((N, H, Nd))
    fYc = np.empty((N, H, Nd))
    scores = np.empty((4, Nd))

    def step(x, nu):
        xn = np.empty_like(x)
        xn[0] = x[0]
        xn[1:N + 1] = PAI.T @ x + nu
        xn[N + 1:] = x[1:K - N]
        return xn

    for nn in range(Nd):
        logSV = logSV0[:, None] + np.cumsum(svshocks[:, :, nn], axis=1)
        sv = np.exp(logSV * 0.5)
        nu = invA @ (sv * z[:, :, nn])
        # linear simulation (ltitr, :322-323)
        x = Xjumpoff.copy()
        for hh in range(H):
            x = step(x, nu[:, hh])
            fY[:, hh, nn] = x[1:N + 1]
        # one-step predictive scores (:326-352)
        muY = PAI.T @ Xjumpoff
        sqrtOmegaY = invA * sv[:, 0][None, :]
        scores[0, nn] = logscore_gaussian(muY, sqrtOmegaY, yrealized, np.sum(logSV[:, 0]))
        if yNatELB > 0:
            scores[1, nn] = logscore_gaussian_censored(muY, sqrtOmegaY, yrealized, elb, ndxYields)
        else:
            scores[1, nn] = scores[0, nn]
        Sx = sqrtOmegaY[ndxYx, :]
        Lx = np.linalg.cholesky(Sx @ Sx.T)
        scores[2, nn] = logscore_gaussian(muY[ndxYx], Lx, yrealized[ndxYx],
                                          2 * np.sum(np.log(np.diag(Lx))))
        Si = sqrtOmegaY[ndxYi, :]
        Li = np.linalg.cholesky(Si @ Si.T)
        if yNatELB > 0:
            scores[3, nn] = logscore_gaussian_censored(muY[ndxYi], Li, yrealized[ndxYi], elb)
        else:
            scores[3, nn] = logscore_gaussian(muY[ndxYi], Li, yrealized[ndxYi])
        # censored simulation (:355-372)
        x = Xjumpoff.copy()
        for hh in range(H):
            x = step(x, nu[:, hh])
            yd = x[1:N + 1].copy()
            m = ndxYields & (yd < elb)
            if m.any():
                yd[m] = elb
                x[1:N + 1] = yd
            fYc[:, hh, nn] = yd
    # RB mean path (:376-379)
    yhat = np.empty((N, H))
    x = Xjumpoff.copy()
    for hh in range(H):
        x = step(x, np.zeros(N))
        yhat[:, hh] = x[1:N + 1]
    return fY, fYc, yhat, scores


def bh_jumpoff(Y, data, p, ndxYIELDS):
    """Xjumpoff of mcmcVARshadowrateBlockHybrid.m:511-520 (Nstates = K + Nyields p):
    [1, Y(end), ..., Y(end-p+1)] of the (shadow-rate) Y, then the actual data's yields
    data(Nobs-(l-1), ndxYIELDS) for l = 1..p."""
    T, N = Y.shape
    ny = np.flatnonzero(ndxYIELDS)
    x = [np.ones(1)] + [Y[T - l] for l in range(1, p + 1)]
    x += [data[data.shape[0] - l, ny] for l in range(1, p + 1)]
    return np.concatenate(x)


def fcst_draw_bh(PAI, invA, logSV0, sqrtPHI, Xjumpoff, yrealized, ndxYields, actualrateBlock,
                 elb, svz, z):
    """One kept draw of mcmcVARshadowrateBlockHybrid.m:550-625 as written: the dense
    companion fcstA on Nstates = K + Nyields p states (:147-159) with PAIshadow / PAIactual
    (:566-574), the simulation with the actual-rate states max(shadow, ELB) (:611-625),
    and the one-step scores (:577-608).

    Xjumpoff: Nstates (bh_jumpoff).  Returns fcstY N x H x Nd (uncensored: the yields are
    floored afterwards, :696-700) and scores 3 x Nd = (fcstLogscoreDraws,
    fcstLogscoreXdraws, fcstLogscoreIdraws)."""
    K, N = PAI.shape
    p = (K - 1) // N
    H, Nd = z.shape[1], z.shape[2]
    ndxYields = np.asarray(ndxYields, bool)
    actual = np.asarray(actualrateBlock, bool)
    ny = np.flatnonzero(ndxYields)
    Nyields = ny.size
    Nstates = K + Nyields * p
    ndxYIELDLAGS = np.concatenate([[False], np.tile(ndxYields, p)])
    fcstA = np.zeros((Nstates, Nstates))
    fcstA[0, 0] = 1.0
    fcstA[1 + N:K, 1:K - N] = np.eye(N * (p - 1))
    fcstA[K + Nyields:, K:K + Nyields * (p - 1)] = np.eye(Nyields * (p - 1))
    ndxfcstActual = K + np.arange(Nyields)
    ndxfcstShadow = 1 + ny
    ndxfcstY = 1 + np.arange(N)
    fcstB = np.zeros((Nstates, N))
    fcstB[ndxfcstY, :] = np.eye(N)
    PAIactual = PAI[ndxYIELDLAGS, :].copy()
    PAIactual[:, ~actual] = 0.0
    PAIshadow = PAI.copy()
    PAIshadow[np.ix_(ndxYIELDLAGS, actual)] = 0.0
    fcstA[np.ix_(ndxfcstY, np.arange(K))] = PAIshadow.T
    fcstA[np.ix_(ndxfcstY, np.arange(K, Nstates))] = PAIactual.T
    logSVshocks = (sqrtPHI @ svz).reshape(N, H, Nd, order="F")
    logSV = logSV0[:, None, None] + np.cumsum(logSVshocks, axis=1)
    fcstSVdraws = np.exp(logSV * 0.5)
    nushocks = fcstSVdraws * z
    ndxYx = ~ndxYields
    yNatELB = int(np.sum(yrealized[ndxYields] <= elb))
    fY = np.empty((N, H, Nd))
    scores = np.empty((3, Nd))
    for nn in range(Nd):
        muY = (fcstA @ Xjumpoff)[ndxfcstY]
        sqrtOmegaY = invA @ np.diag(fcstSVdraws[:, 0, nn])
        if yNatELB > 0:
            scores[0, nn] = logscore_gaussian_censored(muY, sqrtOmegaY, yrealized, elb, ndxYields)
        else:
            scores[0, nn] = logscore_gaussian(muY, sqrtOmegaY, yrealized, np.sum(logSV[:, 0, nn]))
        Sx = sqrtOmegaY[ndxYx, :]
        Lx = np.linalg.cholesky(Sx @ Sx.T)
        scores[1, nn] = logscore_gaussian(muY[ndxYx], Lx, yrealized[ndxYx],
                                          2 * np.sum(np.log(np.diag(Lx))))
        Si = sqrtOmegaY[ndxYields, :]
        Li = np.linalg.cholesky(Si @ Si.T)
        if yNatELB > 0:
            scores[2, nn] = logscore_gaussian_censored(muY[ndxYields], Li, yrealized[ndxYields], elb)
        else:
            scores[2, nn] = logscore_gaussian(muY[ndxYields], Li, yrealized[ndxYields])
        x = Xjumpoff.copy()
        theseShocks = invA @ nushocks[:, :, nn]
        for hh in range(H):
            xd = fcstA @ x + fcstB @ theseShocks[:, hh]
            fY[:, hh, nn] = xd[ndxfcstY]
            x = xd
            x[ndxfcstActual] = np.maximum(x[ndxfcstShadow], elb)
    return fY, scores


def hybrid_jumpoff(Y, data, p, ndxSHADOWRATE, elb):
    """Xjumpoff of mcmcVARhybridGibbs.m:111-121, 531-536 (Nstates = Kshadow + Ns p):
    [1, Y(end), ..., Y(end-p+1)] of the chain's (shadow-rate) Y, then
    XjumpoffActualYieldLags = data(Nobs-(l-1), ndxSHADOWRATE) floored at the ELB."""
    T, N = Y.shape
    s = np.asarray(ndxSHADOWRATE, int)
    x = [np.ones(1)] + [Y[T - l] for l in range(1, p + 1)]
    x += [np.maximum(data[data.shape[0] - l, s], elb) for l in range(1, p + 1)]
    return np.concatenate(x)


def fcst_draw_hybrid(PAI, invA, logSV0, sqrtPHI, Xjumpoff, yrealized, ndxYields, ndxSHADOWRATE, elb, svz, z):
    """One kept draw of mcmcVARhybridGibbs.m:566-635 as written: the dense companion on
    Nstates = Kshadow + Ns p states (:160-172) with fcstA(ndxfcstY, :) = PAI' (:587), the
    simulation with the actual-rate states max(shadow, ELB) (:623-635) and the one-step scores
    (:590-620).  PAI (Kshadow + Ns p) x N.  Returns fcstY N x H x Nd (uncensored; the yields
    are floored afterwards, :707-711) and scores 3 x Nd = (fcstLogscoreDraws,
    fcstLogscoreXdraws, fcstLogscoreIdraws)."""
    Kx, N = PAI.shape
    s = np.asarray(ndxSHADOWRATE, int)
    Ns = s.size
    p = (Kx - 1) // (N + Ns)
    K = 1 + N * p
    H, Nd = z.shape[1], z.shape[2]
    ndxYields = np.asarray(ndxYields, bool)
    Nstates = K + Ns * p
    fcstA = np.zeros((Nstates, Nstates))
    fcstA[0, 0] = 1.0
    fcstA[1 + N:K, 1:K - N] = np.eye(N * (p - 1))
    fcstA[K + Ns:, K:K + Ns * (p - 1)] = np.eye(Ns * (p - 1))
    ndxfcstActual = K + np.arange(Ns)
    ndxfcstShadow = 1 + s
    ndxfcstY = 1 + np.arange(N)
    fcstB = np.zeros((Nstates, N))
    fcstB[ndxfcstY, :] = np.eye(N)
    fcstA[ndxfcstY, :] = PAI.T
    logSVshocks = (sqrtPHI @ svz).reshape(N, H, Nd, order="F")
    logSV = logSV0[:, None, None] + np.cumsum(logSVshocks, axis=1)
    fcstSVdraws = np.exp(logSV * 0.5)
    nushocks = fcstSVdraws * z
    ndxYx = ~ndxYields
    yNatELB = int(np.sum(yrealized[ndxYields] <= elb))
    fY = np.empty((N, H, Nd))
    scores = np.empty((3, Nd))
    for nn in range(Nd):
        muY = (fcstA @ Xjumpoff)[ndxfcstY]
        sqrtOmegaY = invA @ np.diag(fcstSVdraws[:, 0, nn])
        if yNatELB > 0:
            scores[0, nn] = logscore_gaussian_censored(muY, sqrtOmegaY, yrealized, elb, ndxYields)
        else:
            scores[0, nn] = logscore_gaussian(muY, sqrtOmegaY, yrealized, np.sum(logSV[:, 0, nn]))
        Sx = sqrtOmegaY[ndxYx, :]
        Lx = np.linalg.cholesky(Sx @ Sx.T)
        scores[1, nn] = logscore_gaussian(muY[ndxYx], Lx, yrealized[ndxYx], 2 * np.sum(np.log(np.diag(Lx))))
        Si = sqrtOmegaY[ndxYields, :]
        Li = np.linalg.cholesky(Si @ Si.T)
        if yNatELB > 0:
            scores[2, nn] = logscore_gaussian_censored(muY[ndxYields], Li, yrealized[ndxYields], elb)
        else:
            scores[2, nn] = logscore_gaussian(muY[ndxYields], Li, yrealized[ndxYields])
        x = Xjumpoff.copy()
        theseShocks = invA @ nushocks[:, :, nn]
        for hh in range(H):
            xd = fcstA @ x + fcstB @ theseShocks[:, hh]
            fY[:, hh, nn] = xd[ndxfcstY]
            x = xd
            x[ndxfcstActual] = np.maximum(x[ndxfcstShadow], elb)
    return fY, scores
