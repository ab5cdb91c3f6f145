"""Host-side model setup: the part of the reference samplers that runs once per
vintage before the Gibbs loop (data matrices, Minnesota prior, priors of the
A, PHI and SV blocks, chain initialisation).  It feeds the device-resident
chain set; the sweep itself runs in libccmm.

Follows mcmcVAR.m:28-206 (identical in mcmcVARshadowrateBlockHybrid.m:30-317
for the parts shared by the models), setShadowYields.m, setMinnesotaMean.m and
the CSV import of doMCMClinear.m:47-60.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def importdata_csv(path):
    """``importdata(<fredblockMD*.csv>)`` (doMCMClinear.m:49-60): returns
    ydates (datenum), ncode, tcode, cumcode, data."""
    with open(path) as fh:
        header = fh.readline().strip().split(",")
    body = np.loadtxt(path, delimiter=",", skiprows=1)
    tcode = body[0, 1:]
    cumcode = body[1, 1:] != 0
    cumcode = cumcode | (tcode == 5)
    return dict(ydates=body[2:, 0], ncode=header[1:], tcode=tcode, cumcode=cumcode,
                data=body[2:, 1:])


_SHADOW_LO = ("FEDFUNDS", "TB3MS", "TB6MS", "GS1", "WUXIASHADOWRATE", "KRIPPNERSHADOWRATE")
_OTHER_LO = ("GS5", "GS10", "GS20", "BAA")


def setShadowYields(ncode, ELBbound):
    """setShadowYields.m:1-13 -> (ndxSHADOWRATE, ndxOTHERYIELDS, ndxYIELDS), 0-based."""
    if ELBbound > 0.25:
        shadow, other = _SHADOW_LO + ("GS5",), ("GS10", "GS20", "BAA")
    else:
        shadow, other = _SHADOW_LO, _OTHER_LO
    s = np.flatnonzero([c in shadow for c in ncode])
    o = np.flatnonzero([c in other for c in ncode])
    return s, o, np.union1d(s, o)


_LEVEL_VARS = frozenset(("CUMFNS", "UNRATE", "WPSFD49207", "PPICMM", "PCEPI", "HOUST", "BAAFFM",
                         "BAA10Y", "BAA", "FEDFUNDS", "TB3MS", "TB6MS", "GS1", "GS5", "GS10", "GS20",
                         "WUXIASHADOWRATE", "KRIPPNERSHADOWRATE"))


def setMinnesotaMean(ncode):
    """setMinnesotaMean.m:1-16 (1 for levels and rates, 0 for growth rates)."""
    return np.array([float(c in _LEVEL_VARS) for c in ncode])


@dataclass
class VARModel:
    """Everything one vintage hands to the device: Y, X and the priors."""
    N: int
    p: int
    K: int
    T: int
    Y: np.ndarray          # T x N
    X: np.ndarray          # T x K   [1, y(t-1), ..., y(t-p)]
    iVdiag: np.ndarray     # K x N   diag(iV) (mcmcVAR.m:186)
    iVb: np.ndarray        # K x N   iVb_prior
    sPHI: np.ndarray       # N x N   (mcmcVAR.m:165)
    dPHI: int              # N + 3   (mcmcVAR.m:164)
    Vol_0mean: np.ndarray  # N       (mcmcVAR.m:168)
    Vol_0vcvsqrt: np.ndarray  # N x N  (mcmcVAR.m:169)
    ARresid: np.ndarray    # (T-1) x N
    Xjumpoff: np.ndarray   # K
    data: np.ndarray       # Nobs x N (sample up to the jump-off)


def build_var(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior=True) -> VARModel:
    """mcmcVAR.m:28-187 for the 1-based jump-off row ``thisT``."""
    data = np.asarray(data0, float)[np.asarray(ydates0) <= ydates0[thisT - 1], :]
    Nobs, N = data.shape
    theta = (0.04, 0.25, 100.0, 2.0) if doRATSprior else (0.05, 0.5, 100.0, 2.0)
    # lags and data matrices (mcmcVAR.m:62-72)
    lagblocks = [data[p - l:Nobs - l, :] for l in range(1, p + 1)]
    X = np.hstack([np.ones((Nobs - p, 1))] + lagblocks)
    Y = data[p:, :].copy()
    T, K = X.shape
    Xjumpoff = np.concatenate([[1.0]] + [data[Nobs - l, :] for l in range(1, p + 1)])
    # AR(1) residual variances (mcmcVAR.m:121-127)
    ARresid = np.empty((T - 1, N))
    for i in range(N):
        Z = np.column_stack([np.ones(T - 1), Y[:-1, i]])
        beta, *_ = np.linalg.lstsq(Z, Y[1:, i], rcond=None)
        ARresid[:, i] = Y[1:, i] - Z @ beta
    s2 = (ARresid ** 2).sum(axis=0) / (T - 2)
    # Minnesota prior (mcmcVAR.m:129-150): coefficient of variable j, lag l in equation i
    lag = np.repeat(np.arange(1, p + 1), N)          # (l, j) with j fastest
    var = np.tile(np.arange(N), p)
    own = var[None, :] == np.arange(N)[:, None]      # N(eq) x N*p
    decay = lag[None, :] ** theta[3]
    pv = np.where(own, theta[0] / decay,
                  (s2[:, None] / s2[var][None, :]) * theta[0] * theta[1] / decay)
    pm = np.where(own & (lag[None, :] == 1), np.asarray(minnesotaPriorMean, float)[:, None], 0.0)
    OMEGA = np.vstack([s2 * theta[2], pv.T])          # K x N
    MU = np.vstack([np.zeros(N), pm.T])
    iVdiag = 1.0 / OMEGA
    dPHI = N + 3
    return VARModel(N=N, p=p, K=K, T=T, Y=Y, X=X, iVdiag=iVdiag, iVb=iVdiag * MU,
                    sPHI=dPHI * 0.15 * np.eye(N) * 12 / np_, dPHI=dPHI, Vol_0mean=np.zeros(N),
                    Vol_0vcvsqrt=10.0 * np.eye(N), ARresid=ARresid, Xjumpoff=Xjumpoff, data=data)


def initial_state(m: VARModel, B: int = 1):
    """PREVdraw at m == 0 (mcmcVAR.m:197-206), replicated over B chains.
    Returns arrays PAI K x N x B, A N x N x B, sqrtht T x N x B, h T x N x B, sqrtPHI N x N x B."""
    sq = np.sqrt(np.vstack([m.ARresid[:1] ** 2, m.ARresid ** 2]))
    PAI, *_ = np.linalg.lstsq(m.X, m.Y, rcond=None)
    rep = lambda a: np.repeat(a[..., None], B, axis=-1)
    return dict(PAI=rep(PAI), A=rep(np.eye(m.N)), sqrtht=rep(sq), h=rep(2 * np.log(sq)),
                sqrtPHI=rep(0.01 * np.eye(m.N)))


def elbT0_of(data, ndxSHADOWRATE, ELBbound, p):
    """goVARshadowrateBlockHybrid.m:131-134 / doMCMCshadowrateBlockHybrid.m:97-100:
    startELB = find(any(data(:,ndxSHADOWRATE) <= ELBbound, 2), 1); elbT0 = startELB - 1 - p."""
    hit = np.any(np.asarray(data)[:, ndxSHADOWRATE] <= ELBbound, axis=1)
    if not hit.any():
        return np.asarray(data).shape[0]  # no ELB observation: empty window
    return int(np.argmax(hit)) + 1 - 1 - p


@dataclass
class BHModel:
    """A vintage of the block-hybrid shadow-rate VAR (mcmcVARshadowrateBlockHybrid.m:30-295)."""
    var: VARModel
    ndxS: np.ndarray          # ndxSHADOWRATE (0-based)
    ndxO: np.ndarray          # ndxOTHERYIELDS (0-based)
    actual_block: np.ndarray  # bool N, actualrateBlock (:80-84: ~ismember(1:N, ndxYIELDS))
    elbT0: int
    elbT: int
    sNaN: np.ndarray          # bool Ns x elbT (:163-171, 192)
    ELB: float
    warn_elbT0: bool          # :203-205 warning condition


def build_bh(thisT, p, np_, data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean,
             ELBbound, elbT0, doRATSprior=True, actualrateBlock=None) -> BHModel:
    """Host setup of mcmcVARshadowrateBlockHybrid.m for the 1-based jump-off ``thisT``:
    the VAR matrices and priors of the actual data (X0, Y0) and the ELB window."""
    m = build_var(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior)
    N, T = m.N, m.T
    ndxS = np.asarray(ndxSHADOWRATE, int)
    ndxO = np.asarray(ndxOTHERYIELDS, int)
    if actualrateBlock is None:  # goVARshadowrateBlockHybrid.m:93
        actual = ~np.isin(np.arange(N), np.union1d(ndxS, ndxO))
    else:
        actual = np.asarray(actualrateBlock, bool)
    cens = np.zeros_like(m.data, dtype=bool)
    cens[:, ndxS] = m.data[:, ndxS] <= ELBbound         # :163-166
    yNaN = cens[p:, :]
    elbT = max(0, T - elbT0)
    if elbT > 0 and np.any(yNaN[:elbT0, ndxS]):
        raise ValueError("something off about elbT0")   # :199-201
    warn = elbT > 0 and not np.any(yNaN[elbT0, ndxS])   # :203-205
    sNaN = yNaN[elbT0:, :][:, ndxS].T if elbT > 0 else np.zeros((ndxS.size, 0), bool)
    return BHModel(var=m, ndxS=ndxS, ndxO=ndxO, actual_block=actual, elbT0=int(elbT0), elbT=elbT,
                   sNaN=sNaN, ELB=float(ELBbound), warn_elbT0=bool(warn))


@dataclass
class HybridModel:
    """A vintage of the hybrid shadow-rate VAR (mcmcVARhybridGibbs.m:33-339): the VAR
    on the shadow-rate data plus the lags of the actual policy rates floored at the ELB."""
    var: VARModel             # X = [1, lags, Xffrlags] (K = Kshadow + Ns p), priors incl. FFRlags
    Kshadow: int              # 1 + N p (:90)
    ndxS: np.ndarray          # ndxSHADOWRATE (0-based)
    elbT0: int
    elbT: int
    sNaN: np.ndarray          # bool Ns x elbT (:206-210)
    ELB: float
    warn_elbT0: bool          # :216-218 warning condition


def build_hybrid(thisT, p, np_, data0, ydates0, ndxSHADOWRATE, minnesotaPriorMean, ELBbound, elbT0,
                 doRATSprior=True) -> HybridModel:
    """Host setup of mcmcVARhybridGibbs.m for the 1-based jump-off ``thisT``."""
    m = build_var(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior)
    theta = (0.04, 0.25, 100.0, 2.0) if doRATSprior else (0.05, 0.5, 100.0, 2.0)
    N, T, data = m.N, m.T, m.data
    Nobs = data.shape[0]
    ndxS = np.asarray(ndxSHADOWRATE, int)
    Ns = ndxS.size
    # Xffrlags: lag l of actual rate s in column (l-1) Ns + s, floored at the ELB (:77-84)
    Xffr = np.hstack([data[p - l:Nobs - l, ndxS] for l in range(1, p + 1)])
    Xffr = np.where(Xffr < ELBbound, ELBbound, Xffr)
    # FFRlags prior (:275-298): Minnesota variance of "variable ndxS(s), lag l" in equation i
    s2 = (m.ARresid ** 2).sum(axis=0) / (T - 2)
    lag = np.repeat(np.arange(1, p + 1), Ns).astype(float)
    var = np.tile(ndxS, p)
    own = var[None, :] == np.arange(N)[:, None]            # N(eq) x Ns p
    decay = lag[None, :] ** theta[3]
    pv = np.where(own, theta[0] / decay, (s2[:, None] / s2[var][None, :]) * theta[0] * theta[1] / decay)
    iVd = np.vstack([m.iVdiag, 1.0 / pv.T])
    iVb = np.vstack([m.iVb, np.zeros((Ns * p, N))])        # prior mean 0 (:276)
    jump = np.concatenate([m.Xjumpoff, np.maximum(np.concatenate(
        [data[Nobs - l, ndxS] for l in range(1, p + 1)]), ELBbound)])  # :117-121
    hv = VARModel(N=N, p=p, K=m.K + Ns * p, T=T, Y=m.Y, X=np.hstack([m.X, Xffr]), iVdiag=iVd,
                  iVb=iVb, sPHI=m.sPHI, dPHI=m.dPHI, Vol_0mean=m.Vol_0mean,
                  Vol_0vcvsqrt=m.Vol_0vcvsqrt, ARresid=m.ARresid, Xjumpoff=jump, data=data)
    cens = np.zeros_like(data, dtype=bool)
    cens[:, ndxS] = data[:, ndxS] <= ELBbound               # :178-187
    yNaN = cens[p:, :]
    elbT = max(0, T - elbT0)
    if elbT > 0 and np.any(yNaN[:elbT0, ndxS]):
        raise ValueError("something off about elbT0")       # :212-214
    warn = elbT > 0 and not np.any(yNaN[elbT0, ndxS])       # :216-218
    sNaN = yNaN[elbT0:, :][:, ndxS].T if elbT > 0 else np.zeros((Ns, 0), bool)
    return HybridModel(var=hv, Kshadow=m.K, ndxS=ndxS, elbT0=int(elbT0), elbT=elbT, sNaN=sNaN,
                       ELB=float(ELBbound), warn_elbT0=bool(warn))
