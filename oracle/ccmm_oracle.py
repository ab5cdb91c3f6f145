"""CPU restatement (numpy/scipy) of the CCMM BVAR-SV Gibbs sweep — the ORACLE.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``.  The product path never uses it.

PARITY UNPINNED.  The reference (Allisterh/CCMMshadowrateVAR-code @ 2025-01-27)
is MATLAB; no MATLAB/Octave exists in this image, and the reference ships no
tests, golden vectors or fixtures.  This file restates the
reference algorithm line by line *as written* (kron-materialised X_j, explicit
inverse of the Cholesky factor, QR with Q for the ELB smoothing weights), with
every ``randn``/``rand`` replaced by a read of a common-random-number (CRN)
array in MATLAB column-major order.  It is pinned only by mathematical
known-answer tests (closed-form conjugate posteriors, KSC mixture identities,
truncated-normal CDF identities) in ``tests/test_oracle.py``.

The stochastic-volatility block ``StochVolKSCcorrsqrt`` and ``getKSC7values``
live in the absent ``em-matlabbox`` submodule (.gitmodules:1-3, commit pin
unknown).  They are restated here from the published algorithm:
Kim, Shephard & Chib (1998) 7-component log-chi2 mixture (Table 4 constants)
and a precision-based (block-tridiagonal Cholesky) joint draw of the
random-walk log-variances h_0..h_T with correlated shocks sqrtPHI.  The CRN
layout of that block is this build's own declaration (``SV_CRN`` below).

Conventions: all matrices use the reference's shapes (Y is T x N, X is T x K,
PAI is K x N, A is N x N unit lower triangular, sqrtht is T x N).  Indices
are 0-based in code, citations are to the 1-based MATLAB source.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
from scipy.linalg import cholesky, solve_triangular
from scipy.special import erfc, erfcinv

EPS = np.finfo(float).eps  # MATLAB eps

# --------------------------------------------------------------------------
# KSC (1998) 7-component mixture approximating log chi2(1)  [getKSC7values, ext]
# --------------------------------------------------------------------------
KSC_PROB = np.array([0.00730, 0.10556, 0.00002, 0.04395, 0.34001, 0.24566, 0.25750])
KSC_MEAN = np.array([-10.12999, -3.97281, -8.56686, 2.77786, 0.61942, 1.79518, -1.08819]) - 1.2704
KSC_VAR = np.array([5.79596, 2.61369, 5.17950, 0.16735, 0.64009, 0.34023, 1.26261])
KSC_VOL = np.sqrt(KSC_VAR)
# getKSC7values(T,N) also returns logy2offset (mcmcVAR.m:173,259); its value is
# in the absent toolbox.  This build declares 1e-3 (configurable everywhere).
LOGY2OFFSET = 1e-3


# --------------------------------------------------------------------------
# Data and configuration helpers
# --------------------------------------------------------------------------
def load_fred_csv(path):
    """importdata() of a fredblockMD20*.csv file (goVARshadowrateBlockHybrid.m:73-86,
    doMCMClinear.m:49-60): row 1 names, row 2 tcode, row 3 cumcode, then
    ``datenum, values...``."""
    with open(path) as fh:
        names = fh.readline().strip().split(",")
    raw = np.genfromtxt(path, delimiter=",", skip_header=1)
    ncode = names[1:]
    tcode = raw[0, 1:]
    cumcode = raw[1, 1:].astype(bool)
    cumcode[tcode == 5] = True
    ydates = raw[2:, 0]
    data = raw[2:, 1:]
    return dict(ncode=ncode, tcode=tcode, cumcode=cumcode, ydates=ydates, data=data)


def set_shadow_yields(ncode, ELBbound):
    """setShadowYields.m:1-13 (0-based index arrays)."""
    if ELBbound > 0.25:
        s = {"FEDFUNDS", "TB3MS", "TB6MS", "GS1", "WUXIASHADOWRATE", "KRIPPNERSHADOWRATE", "GS5"}
        o = {"GS10", "GS20", "BAA"}
    else:
        s = {"FEDFUNDS", "TB3MS", "TB6MS", "GS1", "WUXIASHADOWRATE", "KRIPPNERSHADOWRATE"}
        o = {"GS5", "GS10", "GS20", "BAA"}
    ndxS = np.array([i for i, c in enumerate(ncode) if c in s], dtype=int)
    ndxO = np.array([i for i, c in enumerate(ncode) if c in o], dtype=int)
    return ndxS, ndxO, np.union1d(ndxS, ndxO)


_MINN_LEVEL = {"CUMFNS", "UNRATE", "WPSFD49207", "PPICMM", "PCEPI", "HOUST", "BAAFFM",
               "BAA10Y", "BAA", "FEDFUNDS", "TB3MS", "TB6MS", "GS1", "GS5", "GS10", "GS20",
               "WUXIASHADOWRATE", "KRIPPNERSHADOWRATE"}


def set_minnesota_mean(ncode):
    """setMinnesotaMean.m:1-16."""
    return np.array([1.0 if c in _MINN_LEVEL else 0.0 for c in ncode])


def elb_t0(data, ndxSHADOWRATE, ELBbound, p):
    """doMCMCshadowrateBlockHybrid.m:97-100 / goVARshadowrateBlockHybrid.m:131-134 (0-based
    count == MATLAB value, since elbT0 is a count of observations)."""
    d = data[:, ndxSHADOWRATE] <= ELBbound
    startELB = int(np.argmax(d.any(axis=1))) + 1  # 1-based find(...,1)
    return startELB - 1 - p


# --------------------------------------------------------------------------
# Model setup (mcmcVAR.m:28-206; mcmcVARshadowrateBlockHybrid.m:30-317)
# --------------------------------------------------------------------------
@dataclass
class Setup:
    N: int
    p: int
    T: int
    K: int
    X: np.ndarray
    Y: np.ndarray
    ARresid: np.ndarray
    iVdiag: np.ndarray  # K x N   diag of iV, equation blocks in columns
    iVb: np.ndarray     # K x N   iVb_prior reshaped
    sPHI: np.ndarray
    dPHI: int
    Vol_0mean: np.ndarray
    Vol_0vcvsqrt: np.ndarray
    Xjumpoff: np.ndarray
    data: np.ndarray
    logy2offset: float = LOGY2OFFSET
    extra: dict = field(default_factory=dict)


def build_lags(data, p):
    """X, Y construction (mcmcVAR.m:62-72)."""
    Nobs, N = data.shape
    lags = np.zeros((Nobs, N * p))
    for l in range(1, p + 1):
        lags[p:, N * (l - 1):N * l] = data[p - l:Nobs - l, :]
    X = np.hstack([np.ones((Nobs - p, 1)), lags[p:, :]])
    Y = data[p:, :].copy()
    return X, Y


def var_setup(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior=True,
              logy2offset=LOGY2OFFSET):
    """mcmcVAR.m:28-187 (thisT is the 1-based row index of the jump-off)."""
    samEnd = ydates0[thisT - 1]
    data = data0[ydates0 <= samEnd, :]
    theta = [0.04, 0.25, 100, 2] if doRATSprior else [0.05, 0.5, 100, 2]
    Nobs, N = data.shape
    X, Y = build_lags(data, p)
    T, K = X.shape
    Klagreg = K - 1
    Xjumpoff = np.zeros(K)
    Xjumpoff[0] = 1
    for l in range(1, p + 1):
        Xjumpoff[1 + (l - 1) * N:1 + l * N] = data[Nobs - l, :]
    # AR(1) residuals (mcmcVAR.m:121-127)
    ARresid = np.full((T - 1, N), np.nan)
    for i in range(N):
        yt0 = np.column_stack([np.ones(T - 1), Y[:-1, i]])
        yt1 = Y[1:, i]
        b = np.linalg.lstsq(yt0, yt1, rcond=None)[0]
        ARresid[:, i] = yt1 - yt0 @ b
    AR_s2 = np.sum(ARresid ** 2, axis=0) / (T - 2)
    # Minnesota prior (mcmcVAR.m:129-150)
    Pi_pm = np.zeros(N * Klagreg)
    Pi_pv = np.zeros(N * Klagreg)
    sigma_const = np.zeros(N)
    co = 0
    for i in range(N):
        sigma_const[i] = AR_s2[i] * theta[2]
        for l in range(1, p + 1):
            for j in range(N):
                if i == j:
                    if l == 1:
                        Pi_pm[co] = minnesotaPriorMean[i]
                    Pi_pv[co] = theta[0] / (l ** theta[3])
                else:
                    Pi_pv[co] = AR_s2[i] / AR_s2[j] * theta[0] * theta[1] / (l ** theta[3])
                co += 1
    OMEGA = np.vstack([sigma_const[None, :], Pi_pv.reshape(N, Klagreg).T])  # K x N
    MU = np.vstack([np.zeros((1, N)), Pi_pm.reshape(N, Klagreg).T])
    iVdiag = 1.0 / OMEGA
    iVb = iVdiag * MU
    dPHI = N + 3
    sPHI = dPHI * (0.15 * np.eye(N)) * 12 / np_
    return Setup(N=N, p=p, T=T, K=K, X=X, Y=Y, ARresid=ARresid, iVdiag=iVdiag, iVb=iVb,
                 sPHI=sPHI, dPHI=dPHI, Vol_0mean=np.zeros(N), Vol_0vcvsqrt=10 * np.eye(N),
                 Xjumpoff=Xjumpoff, data=data, logy2offset=logy2offset)


def init_state(su: Setup):
    """Chain initialisation at m == 0 (mcmcVAR.m:197-206)."""
    sqrtht = np.sqrt(np.vstack([su.ARresid[:1, :] ** 2, su.ARresid ** 2]))
    return dict(A=np.eye(su.N), PAI=np.linalg.lstsq(su.X, su.Y, rcond=None)[0],
                sqrtht=sqrtht, h=2 * np.log(sqrtht), sqrtPHI=math.sqrt(1e-4) * np.eye(su.N),
                Y=su.Y.copy(), X=su.X.copy())


# --------------------------------------------------------------------------
# CRN layout of one sweep (SURVEY.md §8a "Per-sweep RNG consumption order")
# --------------------------------------------------------------------------
def crn_sizes(N, K, T, dPHI):
    """Return the ordered list of (name, shape) CRN blocks for one linear sweep.

    1. zPAI randn(K,N)        CTA.m:58 / CTAsys.m:58
    2. zA   N(N-1)/2 normals  mcmcVAR.m:251  (19 calls randn(ii-1,1), concatenated)
    3. uSV  rand(N,T)         SV mixture indicators  (this build's declaration)
    4. zSV  randn(N,T+1)      SV joint draw of h_0..h_T (this build's declaration)
    5. zPHI randn(N,T+dPHI)   mcmcVAR.m:268
    """
    return [("zPAI", (K, N)), ("zA", (N * (N - 1) // 2,)), ("uSV", (N, T)),
            ("zSV", (N, T + 1)), ("zPHI", (N, T + dPHI))]


def draw_crn(rng, N, K, T, dPHI):
    out = {}
    for name, shape in crn_sizes(N, K, T, dPHI):
        out[name] = rng.random(shape) if name.startswith("u") else rng.standard_normal(shape)
    return out


# --------------------------------------------------------------------------
# CTA / CTAsys (CTA.m:57-98; CTAsys.m:57-108)
# --------------------------------------------------------------------------
def _cta_post(Xj, Yj, iVd, iVbj, zj, K, force_qr=False):
    """Posterior moments and draw for one equation (CTA.m:72-96).  force_qr: take the QR
    branch (CTA.m:80-92) as if chol had failed (test hook for the device fallback)."""
    Ik = np.eye(K)
    iVpost = np.diag(iVd) + Xj.T @ Xj
    status = 0
    try:
        if force_qr:
            raise np.linalg.LinAlgError("forced")
        L = np.linalg.cholesky(iVpost)
        Vchol = solve_triangular(L, Ik, lower=True).T  # (iVchol_post \ Ik)'
    except np.linalg.LinAlgError:  # Kailath fast-array QR fallback (CTA.m:80-92)
        status = 1
        iVchol = np.linalg.cholesky(np.diag(iVd))
        R = np.linalg.qr(np.hstack([iVchol, Xj.T]).T, mode="r")
        L = np.triu(R).T[:K, :K]
        Vchol = solve_triangular(L, Ik, lower=True).T
    Vpost = Vchol @ Vchol.T
    b = Vpost @ (iVbj + Xj.T @ Yj)
    return b + Vchol @ zj, status, np.sqrt(np.diag(Vpost))


def cta(Y, X, N, K, A, sqrtht, iVdiag, iVb, PAI, z, return_sd=False, force_qr=False):
    """CTA.m:57-98 as written (kron-materialised X_j, explicit inverse).
    return_sd: also return the posterior sd of each coefficient (K x N), the
    scale of the parity metric |delta| / max(|x|, sd_post)."""
    PAI = np.array(PAI, dtype=float, copy=True)
    sd = np.zeros((K, N))
    status = 0
    for j in range(N):
        PAI[:, j] = 0.0
        lam = sqrtht[:, j:].ravel(order="F")
        Yj = ((Y - X @ PAI) @ A[j:, :].T).ravel(order="F") / lam
        Xj = np.kron(A[j:, j][:, None], X) / lam[:, None]
        PAI[:, j], s, sd[:, j] = _cta_post(Xj, Yj, iVdiag[:, j], iVb[:, j], z[:, j], K, force_qr)
        status |= s
    if return_sd:
        return PAI, status, sd
    return PAI, status


def cta_sys(Y, XX, N, K, T, A, sqrtht, iVdiag, iVb, PAI, z, return_sd=False, force_qr=False):
    """CTAsys.m:57-108 as written; XX is T x K x N (one design per equation)."""
    PAI = np.array(PAI, dtype=float, copy=True)
    sd = np.zeros((K, N))
    status = 0
    for j in range(N):
        XPAI = np.empty((T, N))
        for jj in range(N):
            XPAI[:, jj] = 0.0 if jj == j else XX[:, :, jj] @ PAI[:, jj]
        lam = sqrtht[:, j:].ravel(order="F")
        Yj = ((Y - XPAI) @ A[j:, :].T).ravel(order="F") / lam
        Xj = np.kron(A[j:, j][:, None], XX[:, :, j]) / lam[:, None]
        PAI[:, j], s, sd[:, j] = _cta_post(Xj, Yj, iVdiag[:, j], iVb[:, j], z[:, j], K, force_qr)
        status |= s
    if return_sd:
        return PAI, status, sd
    return PAI, status


def cta_sys_aswitching(Y, XX, N, K, T, A, Aelb, atELB, sqrtht, iVdiag, iVb, PAI, z, return_sd=False,
                       force_qr=False):
    """CTAsysAswitching.m:57-110 as written: per equation the kron-materialised designs of the
    months at the ELB (Aelb) stacked over those away from it (A), explicit inverse."""
    PAI = np.array(PAI, dtype=float, copy=True)
    at = np.asarray(atELB, bool)
    sd = np.zeros((K, N))
    status = 0
    for j in range(N):
        XPAI = np.empty((T, N))
        for jj in range(N):
            XPAI[:, jj] = 0.0 if jj == j else XX[:, :, jj] @ PAI[:, jj]
        lam_at = sqrtht[at, j:].ravel(order="F")
        lam_aw = sqrtht[~at, j:].ravel(order="F")
        YX = Y - XPAI
        Yj = np.concatenate([(YX[at] @ Aelb[j:, :].T).ravel(order="F") / lam_at,
                             (YX[~at] @ A[j:, :].T).ravel(order="F") / lam_aw])
        Xj = np.vstack([np.kron(Aelb[j:, j][:, None], XX[at, :, j]) / lam_at[:, None],
                        np.kron(A[j:, j][:, None], XX[~at, :, j]) / lam_aw[:, None]])
        PAI[:, j], s, sd[:, j] = _cta_post(Xj, Yj, iVdiag[:, j], iVb[:, j], z[:, j], K, force_qr)
        status |= s
    if return_sd:
        return PAI, status, sd
    return PAI, status


def cta_syrk(Y, X, N, K, A, sqrtht, iVdiag, iVb, PAI, z):
    """CTA.m:57-98 in the algorithmic form the device uses: per equation
    the weighted Gram X' diag(w) X + diag(iV_j) (no kron materialisation), Cholesky and
    two triangular solves.  Equal to ``cta`` in exact arithmetic; the second CPU baseline
    line of bench.py."""
    PAI = np.array(PAI, dtype=float, copy=True)
    ih2 = 1.0 / sqrtht ** 2
    for j in range(N):
        PAI[:, j] = 0.0
        E = Y - X @ PAI
        w = ih2[:, j:] @ (A[j:, j] ** 2)
        v = ((E @ A[j:, :].T) * ih2[:, j:]) @ A[j:, j]
        G = X.T @ (X * w[:, None])
        G[np.diag_indices(K)] += iVdiag[:, j]
        L = np.linalg.cholesky(G)
        y = solve_triangular(L, iVb[:, j] + X.T @ v, lower=True)
        PAI[:, j] = solve_triangular(L.T, y + z[:, j], lower=False)
    return PAI, 0


def cta_sys_syrk(Y, Xs, N, K, T, A, sqrtht, iVdiag, iVb, PAI, z, return_sd=False):
    """CTAsys.m:57-108 in the algorithmic (weighted-SYRK) form, for systems where the
    as-written kron form is out of reach (S120: K = 1441, N = 120, X_j up to 1 GB).
    Xs: list of N designs (T x K each; equations sharing a slab may share the array).
    XPAI (CTAsys.m:67-73: X_jj PAI(:,jj) of every other equation, with the columns < j
    already redrawn) is kept up to date column by column instead of recomputed per j:
    the same values.  Per equation: G = X_j' diag(w) X_j + diag(iV_j), rhs = iVb_j + X_j' v
    (SURVEY.md §3.4 identity), Cholesky, two triangular solves (CTA.m:95-96 with
    Vchol = L^-T).  return_sd: posterior sd per coefficient (sqrt diag G^-1)."""
    PAI = np.array(PAI, dtype=float, copy=True)
    sd = np.zeros((K, N))
    ih2 = 1.0 / sqrtht ** 2
    XPAI = np.column_stack([Xs[jj] @ PAI[:, jj] for jj in range(N)])
    for j in range(N):
        E = Y - XPAI
        E[:, j] = Y[:, j]
        w = ih2[:, j:] @ (A[j:, j] ** 2)
        v = ((E @ A[j:, :].T) * ih2[:, j:]) @ A[j:, j]
        Xj = Xs[j]
        G = Xj.T @ (Xj * w[:, None])
        G[np.diag_indices(K)] += iVdiag[:, j]
        L = np.linalg.cholesky(G)
        y = solve_triangular(L, iVb[:, j] + Xj.T @ v, lower=True)
        PAI[:, j] = solve_triangular(L.T, y + z[:, j], lower=False)
        XPAI[:, j] = Xj @ PAI[:, j]
        if return_sd:
            Li = solve_triangular(L, np.eye(K), lower=True)
            sd[:, j] = np.sqrt(np.einsum("ik,ik->k", Li, Li))
    if return_sd:
        return PAI, 0, sd
    return PAI, 0


def cta_post_moments_syrk(Y, X, N, K, A, sqrtht, iVdiag, iVb, PAI, j):
    """Algebraic (weighted-SYRK) form of equation j's posterior precision and rhs,
    used only by tests to cross-check the kron form (SURVEY.md §3.4 identity)."""
    PAI = PAI.copy()
    PAI[:, j] = 0
    E = Y - X @ PAI
    ih2 = 1.0 / sqrtht[:, j:] ** 2
    w = ih2 @ (A[j:, j] ** 2)
    EA = E @ A[j:, :].T
    v = (EA * ih2) @ A[j:, j]
    return np.diag(iVdiag[:, j]) + X.T @ (X * w[:, None]), iVb[:, j] + X.T @ v


# --------------------------------------------------------------------------
# A-matrix block (mcmcVAR.m:236-254), flat prior (mcmcVAR.m:153-161)
# --------------------------------------------------------------------------
def a_step(RESID, sqrtht, zA):
    T, N = RESID.shape
    A = np.eye(N)
    off = 0
    for ii in range(1, N):
        y = RESID[:, ii] / sqrtht[:, ii]
        Xa = RESID[:, :ii] / sqrtht[:, ii:ii + 1]
        ZZ = Xa.T @ Xa
        Zz = Xa.T @ y
        U = cholesky(ZZ, lower=False)
        tilde = solve_triangular(U.T, Zz, lower=True)
        alpha = solve_triangular(U, tilde + zA[off:off + ii], lower=False)
        off += ii
        A[ii, :ii] = -alpha
    invA = solve_triangular(A, np.eye(N), lower=True)
    return A, invA


def a_step_sd(RESID, sqrtht):
    """Posterior sd of the free A entries (sqrt diag of inv(ZZ), flat prior) as an
    N x N lower matrix (1 elsewhere): the scale of the A parity metric."""
    T, N = RESID.shape
    sd = np.ones((N, N))
    for ii in range(1, N):
        Xa = RESID[:, :ii] / sqrtht[:, ii:ii + 1]
        sd[ii, :ii] = np.sqrt(np.diag(np.linalg.inv(Xa.T @ Xa)))
    return sd


# --------------------------------------------------------------------------
# SV block: restatement of StochVolKSCcorrsqrt (ext, em-matlabbox)
# --------------------------------------------------------------------------
def ksc_indicators(y, hprev, u):
    """7-component mixture indicators (1-based, int8) for each cell.

    For cell (i,t): kernel_k = q_k/vol_k * exp(-0.5*((y-h-mean_k)/vol_k)^2),
    cdf_k = cumsum(kernel)/sum(kernel), cdf_7 := 1, s = 1 + #{k : u > cdf_k}.
    """
    e = (y[..., None] - hprev[..., None] - KSC_MEAN) / KSC_VOL
    ker = KSC_PROB / KSC_VOL * np.exp(-0.5 * e * e)
    cdf = np.cumsum(ker, axis=-1)
    cdf = cdf / cdf[..., -1:]
    cdf[..., -1] = 1.0
    return (1 + np.sum(u[..., None] > cdf, axis=-1)).astype(np.int8)


def sv_separators(T):
    """Separator blocks of the partitioned SV sampler over the T+1 blocks h_0..h_T.

    P = clamp((T+1) // 8, 1, 16) segments; separator k (k = 1..P-1) is block
    floor(k (T+1) / P) - 1.  Segment k's interior is the open range between
    separators k-1 and k (separator 0 = -1, separator P = T+1)."""
    nb = T + 1
    P = max(1, min(16, nb // 8))
    return [(k * nb) // P - 1 for k in range(1, P)]


def sv_precision(obs, ir, sqrtPHI, h0mean, h0vcvsqrt):
    """Blocks of the posterior precision / linear term of x = [h_0; ...; h_T].

    Model: y_t = h_t + mean_{s_t} + eps_t, eps_t ~ N(0, diag(var_{s_t})),
    h_t = h_{t-1} + sqrtPHI e_t, h_0 ~ N(h0mean, V0), V0 = h0vcvsqrt h0vcvsqrt'.
    Returns D (T+1 x N x N diagonal blocks), b (T+1 x N), Q = PHI^{-1}; the
    off-diagonal block between t and t+1 is -Q."""
    N, T = obs.shape
    Q = np.linalg.inv(sqrtPHI @ sqrtPHI.T)
    V0inv = np.linalg.inv(h0vcvsqrt @ h0vcvsqrt.T)
    D = np.empty((T + 1, N, N))
    b = np.empty((T + 1, N))
    D[0] = V0inv + Q
    b[0] = V0inv @ h0mean
    for t in range(1, T + 1):
        D[t] = (Q if t == T else 2 * Q) + np.diag(ir[:, t - 1])
        b[t] = obs[:, t - 1] * ir[:, t - 1]
    return D, b, Q


def sv_draw_sequential(D, b, Q, z):
    """x = P^{-1} b + L^{-T} z with L the time-ordered block Cholesky factor
    (the declared convention for N > 32; for N <= 32 a cross-check of the moments)."""
    T1, N = b.shape
    Ld = np.empty_like(D)
    w = np.empty_like(b)
    Ld[0] = np.linalg.cholesky(D[0])
    w[0] = solve_triangular(Ld[0], b[0], lower=True)
    Lo = np.empty_like(D)
    for t in range(1, T1):
        Lo[t] = -solve_triangular(Ld[t - 1], Q, lower=True).T
        Ld[t] = np.linalg.cholesky(D[t] - Lo[t] @ Lo[t].T)
        w[t] = solve_triangular(Ld[t], b[t] - Lo[t] @ w[t - 1], lower=True)
    x = np.empty_like(b)
    x[T1 - 1] = solve_triangular(Ld[T1 - 1].T, w[T1 - 1] + z[:, T1 - 1], lower=False)
    for t in range(T1 - 2, -1, -1):
        x[t] = solve_triangular(Ld[t].T, w[t] + z[:, t] - Lo[t + 1].T @ x[t + 1], lower=False)
    return x


def sv_draw_partitioned(D, b, Q, z, seps=None):
    """x = P^{-1} b + Pi' L^{-T} z, L the block Cholesky factor of the precision in
    the partitioned order Pi: segment interiors (each in time order), then the
    separators (time order).  z column t belongs to block t.

    Eliminating an interior block t (factor C_t = chol(D~_t), w_t = C_t^{-1} b~_t)
    touches at most two remaining blocks: its successor nxt (coupling M_{t,nxt} = -Q)
    and the segment's left separator s (fill coupling M_{t,s}):
        X1 = C_t^{-1} M_{t,nxt},  X2 = C_t^{-1} M_{t,s}
        D~_nxt -= X1'X1, b~_nxt -= X1'w;   D~_s -= X2'X2, b~_s -= X2'w
        M_{s,nxt} = -X2'X1
    The separators then form a block-tridiagonal system, eliminated in time order.
    Back substitution: x_t = C_t^{-T}(w_t + z_t - C_t^{-1} sum_nbr M_{t,nbr} x_nbr),
    where inside a segment g_t = M_{t,s} x_s obeys g_first = -Q x_s,
    g_{t+1} = Q C_t^{-T} C_t^{-1} g_t."""
    T1, N = b.shape
    if seps is None:
        seps = sv_separators(T1 - 1)
    bounds = [-1] + list(seps) + [T1]
    C = np.empty_like(D)
    w = np.empty_like(b)
    Dsep = {s: D[s].copy() for s in seps}
    bsep = {s: b[s].copy() for s in seps}
    Msep = {}
    negQ = -Q
    for k in range(1, len(bounds)):
        left = bounds[k - 1] if k > 1 else None
        first = bounds[k - 1] + 1
        last = bounds[k] - 1
        Dc, bc = D[first].copy(), b[first].copy()
        Mfill = negQ if left is not None else None  # M_{t,left}
        for t in range(first, last + 1):
            Ct = np.linalg.cholesky(Dc)
            wt = solve_triangular(Ct, bc, lower=True)
            C[t], w[t] = Ct, wt
            nxt = t + 1 if t + 1 < T1 else None
            X1 = solve_triangular(Ct, negQ, lower=True) if nxt is not None else None
            if nxt is not None:
                if t < last:
                    Dc = D[nxt] - X1.T @ X1
                    bc = b[nxt] - X1.T @ wt
                else:
                    Dsep[nxt] -= X1.T @ X1
                    bsep[nxt] -= X1.T @ wt
            if left is not None:
                X2 = solve_triangular(Ct, Mfill, lower=True)
                Dsep[left] -= X2.T @ X2
                bsep[left] -= X2.T @ wt
                if nxt is not None:
                    Mln = -X2.T @ X1  # M_{left, nxt}
                    if t < last:
                        Mfill = Mln.T
                    else:
                        Msep[left] = Mln  # M_{left, right}
    for i, s in enumerate(seps):
        Ct = np.linalg.cholesky(Dsep[s])
        wt = solve_triangular(Ct, bsep[s], lower=True)
        C[s], w[s] = Ct, wt
        if i + 1 < len(seps):
            X1 = solve_triangular(Ct, Msep[s], lower=True)
            s2 = seps[i + 1]
            Dsep[s2] -= X1.T @ X1
            bsep[s2] -= X1.T @ wt
    x = np.empty_like(b)
    for i in range(len(seps) - 1, -1, -1):
        s = seps[i]
        r = w[s] + z[:, s]
        if i + 1 < len(seps):
            r = r - solve_triangular(C[s], Msep[s] @ x[seps[i + 1]], lower=True)
        x[s] = solve_triangular(C[s].T, r, lower=False)
    for k in range(1, len(bounds)):
        left = bounds[k - 1] if k > 1 else None
        first, last = bounds[k - 1] + 1, bounds[k] - 1
        g = {}
        if left is not None:
            gt = negQ @ x[left]
            for t in range(first, last + 1):
                g[t] = gt
                gt = Q @ solve_triangular(C[t].T, solve_triangular(C[t], gt, lower=True), lower=False)
        for t in range(last, first - 1, -1):
            acc = np.zeros(N)
            if t + 1 < T1:
                acc = acc + negQ @ x[t + 1]
            if left is not None:
                acc = acc + g[t]
            x[t] = solve_triangular(C[t].T, w[t] + z[:, t] - solve_triangular(C[t], acc, lower=True),
                                    lower=False)
    return x


def sv_ksc_corrsqrt(y, hprev, sqrtPHI, h0mean, h0vcvsqrt, u, z):
    """Joint draw of log variances with correlated random-walk shocks.

    y, hprev: N x T (logy2', Vol_states').  Model: y_t = h_t + mean_{s_t} + eps_t,
    eps_t ~ N(0, diag(var_{s_t})); h_t = h_{t-1} + sqrtPHI e_t; h_0 ~ N(h0mean, V0),
    V0 = h0vcvsqrt h0vcvsqrt'.  Posterior precision of x = [h_0; ...; h_T] is
    block tridiagonal; x = P^{-1} b + Pi' L^{-T} z with L the block Cholesky factor
    in the partitioned order of ``sv_draw_partitioned`` for N <= 32 and in time order
    (``sv_draw_sequential``, Pi = I) for N > 32 (declared conventions: the reference's
    sampler lives in the absent em-matlabbox; the GPU follows the same split,
    ccmm_svpart.hip / ccmm_bign.hip k_sv_big).  z is N x (T+1), column t for block t.
    Returns h (N x T), h0 (N), shocks (N x T, h_t - h_{t-1}), indicators (N x T int8).
    """
    kai = ksc_indicators(y, hprev, u)
    obs = y - KSC_MEAN[kai - 1]
    ir = 1.0 / KSC_VAR[kai - 1]
    D, b, Q = sv_precision(obs, ir, sqrtPHI, h0mean, h0vcvsqrt)
    x = sv_draw_partitioned(D, b, Q, z) if y.shape[0] <= 32 else sv_draw_sequential(D, b, Q, z)
    h = x[1:].T.copy()
    shocks = (x[1:] - x[:-1]).T.copy()
    return h, x[0].copy(), shocks, kai


# --------------------------------------------------------------------------
# PHI inverse-Wishart block (mcmcVAR.m:268-274)
# --------------------------------------------------------------------------
def phi_iw(eta, sPHI, Zdraw):
    Lpost = cholesky(sPHI + eta.T @ eta, lower=True)
    R = cholesky(Zdraw @ Zdraw.T, lower=False)
    sq = solve_triangular(R.T, Lpost.T, lower=True).T  # Lpost / R
    PHI = sq @ sq.T
    return cholesky(PHI, lower=True), PHI


def vech_lower(M):
    """PHI_((tril(PHI_))~=0): lower triangle, column-major (mcmcVAR.m:290)."""
    N = M.shape[0]
    return np.concatenate([M[j:, j] for j in range(N)])


# --------------------------------------------------------------------------
# One linear BVAR-SV sweep (mcmcVAR.m:211-274)
# --------------------------------------------------------------------------
def linear_sweep(st, su: Setup, crn, cta_form="kron", force_qr=False):
    """cta_form: "kron" = CTA.m as written; "syrk" = the algorithmic form (cta_syrk); "mirror" =
    the device's operation order up to the factorisation (oracle/cta_mirror.py).
    force_qr: every equation takes CTA.m's QR branch (kron form only)."""
    N, K, T = su.N, su.K, su.T
    if cta_form == "kron":
        PAI, status = cta(su.Y, su.X, N, K, st["A"], st["sqrtht"], su.iVdiag, su.iVb, st["PAI"],
                          crn["zPAI"], force_qr=force_qr)
    elif cta_form == "mirror":
        from . import cta_mirror
        PAI = cta_mirror.cta(su.Y, su.X, N, K, st["A"], st["sqrtht"], su.iVdiag, su.iVb, st["PAI"], crn["zPAI"])
        status = 0
    else:
        PAI, status = cta_syrk(su.Y, su.X, N, K, st["A"], st["sqrtht"], su.iVdiag, su.iVb,
                               st["PAI"], crn["zPAI"])
    RESID = su.Y - su.X @ PAI
    A, invA = a_step(RESID, st["sqrtht"], crn["zA"])
    logy2 = np.log((RESID @ A.T) ** 2 + su.logy2offset)
    h, h0, shocks, kai = sv_ksc_corrsqrt(logy2.T, st["h"].T, st["sqrtPHI"], su.Vol_0mean,
                                        su.Vol_0vcvsqrt, crn["uSV"], crn["zSV"])
    h = h.T
    sqrtht = np.exp(h / 2)
    sqrtPHI, PHI = phi_iw(shocks.T, su.sPHI, crn["zPHI"])
    return dict(A=A, invA=invA, PAI=PAI, sqrtht=sqrtht, h=h, sqrtPHI=sqrtPHI, PHI=PHI,
                RESID=RESID, kai=kai.T, h0=h0, status=status, Y=st["Y"], X=st["X"])


# --------------------------------------------------------------------------
# drawTruncNormal (drawTruncNormal.m:31-86)
# --------------------------------------------------------------------------
def draw_trunc_normal(mu, sqrtVCV, elb, u):
    """Returns (draw, flags): bit0 = sigma > tol branch, bit1 = PHIbar > eps branch."""
    tol = 1e-10
    s = abs(sqrtVCV)
    if s > tol:
        ub = (elb - mu) / s
        PHIbar = 0.5 * erfc(-math.sqrt(0.5) * ub)
        if PHIbar > EPS:
            zz = -math.sqrt(2.0) * erfcinv(2.0 * u * PHIbar)
            fl = 3
        else:
            zz = ub
            fl = 1
        return mu + s * zz, fl
    return mu, 0


# --------------------------------------------------------------------------
# gibbsdrawShadowrates (gibbsdrawShadowrates.m:1-245) as written
# --------------------------------------------------------------------------
def gibbsdraw_shadowrates(Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, elbBound, Ndraws,
                          burnin, udraws, return_flags=False):
    """Y Ny x T; STATE0 K; YHAT0 Ny x T or None; ndxS bool Ny; sNaN bool Ns x T;
    C K x K; Psi K x Ny; SVol Ny x T; udraws Ns x T x (burnin+Ndraws)."""
    Y = np.array(Y, dtype=float, copy=True)
    Ny, T = Y.shape
    ndxS = np.asarray(ndxS, dtype=bool)
    ndxX = ~ndxS
    S = Y[ndxS, :].copy()
    Ns = int(ndxS.sum())
    draws = np.full((Ns, T, Ndraws), np.nan)
    Nstate = Ny * p
    NNstate = Nstate + 1
    Nx = Ny - Ns
    H = np.zeros((Ny, NNstate))
    H[:, 1:1 + Ny] = np.eye(Ny)
    Nw = Psi.shape[1]
    if Nw != Ny:
        raise ValueError("dimension mismatch")
    psi = Psi[1:1 + Ny, :]
    PSIt = np.einsum("ij,jt->ijt", psi, SVol)  # psi * diag(SVol(:,t))
    J = np.full((Ns, Nstate + Nx, T), np.nan)
    sqrtOm = np.full((Ns, Ns, T), np.nan)
    cc = C[1:, 1:]
    Cp = np.empty((Nstate, Nstate, p + 1))
    Cp[:, :, 0] = np.eye(Nstate)
    for k in range(p):
        Cp[:, :, k + 1] = cc @ Cp[:, :, k]
    Cp = Cp[:, :Ny, :]
    # smoothing weights (gibbsdrawShadowrates.m:74-95)
    t = 0
    for t in range(1, T - p + 1):
        if sNaN[:, t - 1].any():
            M = np.zeros((Nstate + Nw, Nw * (p + 1)))
            for j in range(p + 1):
                M[:Nstate, Nw * j:Nw * (j + 1)] = Cp[:, :, p - j] @ PSIt[:, :, t - 1 + j]
            M[Nstate:Nstate + Nx, :Nw] = PSIt[ndxX, :, t - 1]
            M[Nstate + Nx:, :Nw] = PSIt[ndxS, :, t - 1]
            R = np.linalg.qr(M.T, mode="r").T
            n1 = Nstate + Nx
            L11 = R[:n1, :n1]
            J[:, :, t - 1] = solve_triangular(L11.T, R[n1:n1 + Ns, :n1].T, lower=False).T
            sqrtOm[:, :, t - 1] = R[n1:n1 + Ns, n1:n1 + Ns]
    if T - p < 1:
        t = 0
    # tail (gibbsdrawShadowrates.m:101-127)
    while t < T:
        t += 1
        if sNaN[:, t - 1].any():
            k = T - t
            Nsig = Ny * k + Nx
            M = np.zeros((Nsig + Ns, Nsig + Ns))
            for j in range(k + 1):
                M[:Nsig, Nw * j:Nw * (j + 1)] = Cp[:Nsig, :, k - j] @ PSIt[:, :, t - 1 + j]
            M[k * Ny:k * Ny + Nx, :Nw] = PSIt[ndxX, :, t - 1]
            M[Nsig:, :Nw] = PSIt[ndxS, :, t - 1]
            R = np.linalg.qr(M.T, mode="r").T
            L11 = R[:Nsig, :Nsig]
            J[:, :, t - 1] = 0.0
            J[:, Ny * (p - k):, t - 1] = solve_triangular(L11.T, R[Nsig:Nsig + Ns, :Nsig].T,
                                                          lower=False).T
            sqrtOm[:, :, t - 1] = R[Nsig:Nsig + Ns, Nsig:Nsig + Ns]
    # conditional weights for Ns > 1 (gibbsdrawShadowrates.m:130-145)
    if Ns > 1:
        sqrtOm1 = np.full((Ns, T), np.nan)
        beta1 = np.full((Ns, Ns - 1, T), np.nan)
        for t in range(T):
            if sNaN[:, t].any():
                vcv = sqrtOm[:, :, t] @ sqrtOm[:, :, t].T
                for s in range(Ns):
                    o = np.arange(Ns) != s
                    b = np.linalg.solve(vcv[np.ix_(o, o)].T, vcv[s, o])
                    beta1[s, :, t] = b
                    sqrtOm1[s, t] = math.sqrt(vcv[s, s] - b @ vcv[o, s])
    Cex1 = C[1:, 1:]
    HC = Cex1[:Ny, :]
    CCpp1 = np.linalg.matrix_power(Cex1, p + 1)
    # deterministic state (gibbsdrawShadowrates.m:157-165) -- note Y0(:,1) = H*STATE0
    Y0 = np.zeros((Ny, T))
    st0 = np.array(STATE0, dtype=float)
    for t in range(T):
        Y0[:, t] = H @ st0
        if YHAT0 is not None:
            Y0[:, t] += YHAT0[:, t]
        st0 = C @ st0
    Ytilde = Y - Y0
    total = burnin + Ndraws
    flags = np.zeros((Ns, T, total), dtype=np.uint8)
    for n in range(total):
        STATElag = np.zeros(Nstate)
        YY = np.hstack([Ytilde, np.zeros((Ny, p))])
        for t in range(T):
            if sNaN[:, t].any():
                Yhat = HC @ STATElag
                Xresid = Ytilde[ndxX, t] - Yhat[ndxX]
                STATEfuture = YY[:, t + p:t:-1]  # columns t+p, ..., t+1 (1-based t+1 offset)
                STATEtilde = STATEfuture.ravel(order="F") - CCpp1 @ STATElag
                Shat = Yhat[ndxS] + Y0[ndxS, t]
                Spost = Shat + J[:, :, t] @ np.concatenate([STATEtilde, Xresid])
                if Ns == 1:
                    S[0, t], flags[0, t, n] = draw_trunc_normal(Spost[0], sqrtOm[0, 0, t],
                                                                elbBound, udraws[0, t, n])
                else:
                    for s in np.nonzero(sNaN[:, t])[0]:
                        o = np.arange(Ns) != s
                        mu = Spost[s] + beta1[s, :, t] @ (S[o, t] - Spost[o])
                        S[s, t], flags[s, t, n] = draw_trunc_normal(mu, sqrtOm1[s, t], elbBound,
                                                                    udraws[s, t, n])
                Y[ndxS, t] = S[:, t]
                Ytilde[:, t] = Y[:, t] - Y0[:, t]
            if t + 1 >= p:
                STATElag = Ytilde[:, t - p + 1:t + 1][:, ::-1].ravel(order="F")
            else:
                STATElag = np.concatenate([Ytilde[:, t], STATElag[:Ny * (p - 1)]])
        if n >= burnin:
            draws[:, :, n - burnin] = S
    if return_flags:
        return draws, flags
    return draws


# --------------------------------------------------------------------------
# gibbsdrawShadowratesB3 (gibbsdrawShadowratesB3.m:1-231) as written
# --------------------------------------------------------------------------
def gibbsdraw_shadowrates_b3(Y, STATE0, ndxS, sNaN, p, A, B, SVol, elbBound, Ndraws, burnin, udraws,
                             return_flags=False):
    """The B3 variant of gibbsdrawShadowrates: the impact matrix B may vary by month (K x Ny x T, or
    K x Ny repeated, :49-51), the VAR runs on Y itself with the intercept in the state (STATElag
    starts at STATE0, :171; Yhat = C A STATElag, :178; no Y0 path).  Y Ny x T; STATE0 K; ndxS bool
    Ny; sNaN bool Ns x T; A K x K; SVol Ny x T; udraws Ns x T x (burnin + Ndraws)."""
    Y = np.array(Y, dtype=float, copy=True)
    Ny, T = Y.shape
    ndxS = np.asarray(ndxS, dtype=bool)
    ndxX = ~ndxS
    S = Y[ndxS, :].copy()
    Ns = int(ndxS.sum())
    draws = np.full((Ns, T, Ndraws), np.nan)
    Nstate = Ny * p
    Nx = Ny - Ns
    B = np.asarray(B, float)
    if B.ndim == 2:  # :49-51
        B = np.repeat(B[:, :, None], T, axis=2)
    Nw = B.shape[1]
    if Nw != Ny:
        raise ValueError("dimension mismatch")
    Bsvol = np.einsum("ijt,jt->ijt", B[1:1 + Ny, :, :], SVol)  # bb(:,:,t) * diag(SVol(:,t)), :58-62
    J = np.full((Ns, Nstate + Nx, T), np.nan)
    sqrtOm = np.full((Ns, Ns, T), np.nan)
    aa = A[1:, 1:]
    Ap = np.empty((Nstate, Nstate, p + 1))
    Ap[:, :, 0] = np.eye(Nstate)
    for k in range(p):
        Ap[:, :, k + 1] = aa @ Ap[:, :, k]
    Ap = Ap[:, :Ny, :]
    t = 0
    for t in range(1, T - p + 1):  # :79-100
        if sNaN[:, t - 1].any():
            M = np.zeros((Nstate + Nw, Nw * (p + 1)))
            for j in range(p + 1):
                M[:Nstate, Nw * j:Nw * (j + 1)] = Ap[:, :, p - j] @ Bsvol[:, :, t - 1 + j]
            M[Nstate:Nstate + Nx, :Nw] = Bsvol[ndxX, :, t - 1]
            M[Nstate + Nx:, :Nw] = Bsvol[ndxS, :, t - 1]
            R = np.linalg.qr(M.T, mode="r").T
            n1 = Nstate + Nx
            J[:, :, t - 1] = solve_triangular(R[:n1, :n1].T, R[n1:n1 + Ns, :n1].T, lower=False).T
            sqrtOm[:, :, t - 1] = R[n1:n1 + Ns, n1:n1 + Ns]
    if T - p < 1:
        t = 0
    while t < T:  # :106-132
        t += 1
        if sNaN[:, t - 1].any():
            k = T - t
            Nsig = Ny * k + Nx
            M = np.zeros((Nsig + Ns, Nsig + Ns))
            for j in range(k + 1):
                M[:Nsig, Nw * j:Nw * (j + 1)] = Ap[:Nsig, :, k - j] @ Bsvol[:, :, t - 1 + j]
            M[k * Ny:k * Ny + Nx, :Nw] = Bsvol[ndxX, :, t - 1]
            M[Nsig:, :Nw] = Bsvol[ndxS, :, t - 1]
            R = np.linalg.qr(M.T, mode="r").T
            J[:, :, t - 1] = 0.0
            J[:, Ny * (p - k):, t - 1] = solve_triangular(R[:Nsig, :Nsig].T, R[Nsig:Nsig + Ns, :Nsig].T,
                                                          lower=False).T
            sqrtOm[:, :, t - 1] = R[Nsig:Nsig + Ns, Nsig:Nsig + Ns]
    if Ns > 1:  # :135-150
        sqrtOm1 = np.full((Ns, T), np.nan)
        beta1 = np.full((Ns, Ns - 1, T), np.nan)
        for t in range(T):
            if sNaN[:, t].any():
                vcv = sqrtOm[:, :, t] @ sqrtOm[:, :, t].T
                for s in range(Ns):
                    o = np.arange(Ns) != s
                    b = np.linalg.solve(vcv[np.ix_(o, o)].T, vcv[s, o])
                    beta1[s, :, t] = b
                    sqrtOm1[s, t] = math.sqrt(vcv[s, s] - b @ vcv[o, s])
    CAA = A[1:1 + Ny, :]                                  # C * A, :153
    AApp1 = np.linalg.matrix_power(A, p + 1)[1:, :]       # :154-155
    total = burnin + Ndraws
    flags = np.zeros((Ns, T, total), dtype=np.uint8)
    for n in range(total):                                # :168-229
        STATElag = np.array(STATE0, dtype=float, copy=True)
        YY = np.hstack([Y, np.zeros((Ny, p))])
        for t in range(T):
            if sNaN[:, t].any():
                Yhat = CAA @ STATElag
                Xresid = Y[ndxX, t] - Yhat[ndxX]
                Shat = Yhat[ndxS]
                STATEtilde = YY[:, t + p:t:-1].ravel(order="F") - AApp1 @ STATElag
                Spost = Shat + J[:, :, t] @ np.concatenate([STATEtilde, Xresid])
                if Ns == 1:
                    S[0, t], flags[0, t, n] = draw_trunc_normal(Spost[0], sqrtOm[0, 0, t], elbBound,
                                                                udraws[0, t, n])
                else:
                    for s in np.nonzero(sNaN[:, t])[0]:
                        o = np.arange(Ns) != s
                        mu = Spost[s] + beta1[s, :, t] @ (S[o, t] - Spost[o])
                        S[s, t], flags[s, t, n] = draw_trunc_normal(mu, sqrtOm1[s, t], elbBound,
                                                                    udraws[s, t, n])
                Y[ndxS, t] = S[:, t]
            if t + 1 >= p:                                # :213-221
                STATElag[1:] = Y[:, t - p + 1:t + 1][:, ::-1].ravel(order="F")
            else:
                STATElag = np.concatenate([[1.0], Y[:, t], STATElag[1:1 + Ny * (p - 1)]])
        if n >= burnin:
            draws[:, :, n - burnin] = S
    if return_flags:
        return draws, flags
    return draws
