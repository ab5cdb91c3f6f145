"""Oracle (CPU restatement) of the block-hybrid shadow-rate sampler
mcmcVARshadowrateBlockHybrid.m — TEST INFRASTRUCTURE ONLY (see ccmm_oracle.py).

PARITY UNPINNED (MATLAB reference, no fixtures).  Follows the reference as
written: CTAsys with per-equation designs (actual-rate X for the macro block,
shadow-rate X for the yield block), the linear A/SV/PHI blocks, then the ELB
step with gibbsdrawShadowrates (QR smoothing weights, 100 burn-in + 1 Gibbs
passes: the ``m < MCMCburnin*.5`` branch, mcmcVARshadowrateBlockHybrid.m:435-437,
forced every sweep — the PS-proposal branch needs the absent em-matlabbox
sampler VARTVPSVprecisionsamplerNaN), and the rebuild of X, Y from the shadow
draws (:501-520).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import ccmm_oracle as O


@dataclass
class BHSetup:
    lin: O.Setup            # Y0/X0 (actual data), priors, T, K, N, p
    Xactual: np.ndarray     # T x K
    actualrateBlock: np.ndarray  # bool N
    ndxS: np.ndarray        # shadow-rate variable indices (0-based)
    ndxSmask: np.ndarray    # bool N
    lagmask: np.ndarray     # bool K: ndxSHADOWRATELAGS (:85)
    Ydata: np.ndarray       # Nobs x N with censored cells zeroed (:163-171)
    elbT0: int
    elbT: int
    sNaN: np.ndarray        # Ns x elbT
    X0: np.ndarray          # K   elb.X0 = X(elbT0+1,:)'
    ELB: float
    gibbsburn: int = 100


def bh_setup(thisT, p, np_, data0, ydates0, ndxS, ndxO, minnesotaPriorMean, ELBbound, elbT0,
             doRATSprior=True, logy2offset=O.LOGY2OFFSET):
    """mcmcVARshadowrateBlockHybrid.m:30-295 (ELB state space :162-220)."""
    lin = O.var_setup(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior, logy2offset)
    N, T, K = lin.N, lin.T, lin.K
    data = lin.data
    ndxY = np.union1d(ndxS, ndxO)
    actual = ~np.isin(np.arange(N), ndxY)
    Smask = np.isin(np.arange(N), ndxS)
    lagmask = np.concatenate([[False], np.tile(Smask, p)])
    Ydata = data.copy()
    sr = Ydata[:, ndxS].copy()
    sr[sr <= ELBbound] = np.nan
    Ydata[:, ndxS] = sr
    yNaNall = np.isnan(Ydata)
    Ydata[yNaNall] = 0.0
    yNaN = yNaNall[p:, :]
    elbT = max(0, T - elbT0)
    if np.any(yNaN[:elbT0, ndxS]):
        raise ValueError("something off about elbT0")
    sNaN = yNaN[elbT0:, :].T[Smask, :]
    return BHSetup(lin=lin, Xactual=lin.X.copy(), actualrateBlock=actual, ndxS=np.asarray(ndxS),
                   ndxSmask=Smask, lagmask=lagmask, Ydata=Ydata, elbT0=elbT0, elbT=elbT,
                   sNaN=sNaN, X0=lin.X[elbT0, :].copy(), ELB=ELBbound)


def bh_crn_sizes(bs: BHSetup):
    lin = bs.lin
    return O.crn_sizes(lin.N, lin.K, lin.T, lin.dPHI) + [
        ("uELB", (len(bs.ndxS), bs.elbT, bs.gibbsburn + 1))]


def bh_draw_crn(rng, bs: BHSetup):
    out = {}
    for name, shape in bh_crn_sizes(bs):
        out[name] = rng.random(shape) if name.startswith("u") else rng.standard_normal(shape)
    return out


def elb_state_space(bs: BHSetup, PAI, invA, sqrtht):
    """mcmcVARshadowrateBlockHybrid.m:400-416: C = elb.A, Psi = elb.B, SVol, Yhatactual."""
    lin = bs.lin
    N, K, p = lin.N, lin.K, lin.p
    PAIactual = PAI[bs.lagmask, :].copy()
    PAIactual[:, ~bs.actualrateBlock] = 0.0
    Yhatactual = (bs.Xactual[bs.elbT0:, bs.lagmask] @ PAIactual).T
    PAIshadow = PAI.copy()
    PAIshadow[np.ix_(bs.lagmask, bs.actualrateBlock)] = 0.0
    C = np.zeros((K, K))
    C[0, 0] = 1.0
    C[1 + N:, 1:1 + N * (p - 1)] = np.eye(N * (p - 1))
    C[1:1 + N, :] = PAIshadow.T
    Psi = np.zeros((K, N))
    Psi[1:1 + N, :] = invA
    SVol = sqrtht[bs.elbT0:, :].T
    return C, Psi, SVol, Yhatactual


def rebuild_XY(bs: BHSetup, shadowrate):
    """mcmcVARshadowrateBlockHybrid.m:480,501-509."""
    lin = bs.lin
    shadowYdata = bs.Ydata.copy()
    shadowYdata[lin.p + bs.elbT0:, bs.ndxS] = shadowrate.T
    X, Y = O.build_lags(shadowYdata, lin.p)
    return X, Y


def bh_init_state(bs: BHSetup):
    st = O.init_state(bs.lin)  # Y = Y0, X = X0 (actual data), mcmcVARshadowrateBlockHybrid.m:310-316
    return st


def bh_sweep(st, bs: BHSetup, crn, return_flags=False, elb_impl="qr"):
    """One sweep m < MCMCburnin/2 of mcmcVARshadowrateBlockHybrid.m:322-523.

    elb_impl: "qr" = gibbsdrawShadowrates as written; "stable" = the same
    conditionals in the residual form of elb_fast.gibbsdraw_shadowrates_stable
    (accurate when the shadow companion matrix is explosive, where the as-written
    Ytilde = Y - Y0 cancels catastrophically); "both" = stable, with the as-written
    draw in out["shadowrate_qr"]."""
    lin = bs.lin
    N, K, T = lin.N, lin.K, lin.T
    Y, X = st["Y"], st["X"]
    XX = np.empty((T, K, N))
    XX[:, :, bs.actualrateBlock] = bs.Xactual[:, :, None]
    XX[:, :, ~bs.actualrateBlock] = X[:, :, None]
    PAI, status = O.cta_sys(Y, XX, N, K, T, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"],
                            crn["zPAI"])
    RESID = np.empty((T, N))
    for jj in range(N):
        RESID[:, jj] = Y[:, jj] - XX[:, :, jj] @ PAI[:, jj]
    A, invA = O.a_step(RESID, st["sqrtht"], crn["zA"])
    logy2 = np.log((RESID @ A.T) ** 2 + lin.logy2offset)
    h, h0, shocks, kai = O.sv_ksc_corrsqrt(logy2.T, st["h"].T, st["sqrtPHI"], lin.Vol_0mean,
                                          lin.Vol_0vcvsqrt, crn["uSV"], crn["zSV"])
    h = h.T
    sqrtht = np.exp(h / 2)
    sqrtPHI, PHI = O.phi_iw(shocks.T, lin.sPHI, crn["zPHI"])
    out = dict(A=A, invA=invA, PAI=PAI, sqrtht=sqrtht, h=h, sqrtPHI=sqrtPHI, PHI=PHI,
               RESID=RESID, kai=kai.T, status=status, Y=Y, X=X)
    if T > bs.elbT0:
        C, Psi, SVol, Yhatactual = elb_state_space(bs, PAI, invA, sqrtht)
        elbY = Y[bs.elbT0:, :].T
        flags = None
        if elb_impl in ("qr", "both"):
            res = O.gibbsdraw_shadowrates(elbY, bs.X0, Yhatactual, bs.ndxSmask, bs.sNaN, lin.p, C,
                                          Psi, SVol, bs.ELB, 1, bs.gibbsburn, crn["uELB"],
                                          return_flags=return_flags)
            draws, flags = (res if return_flags else (res, None))
            out["shadowrate_qr"] = draws[:, :, 0]
        if elb_impl in ("stable", "both"):
            from .elb_fast import gibbsdraw_shadowrates_stable
            draws, sflags = gibbsdraw_shadowrates_stable(elbY, bs.X0, Yhatactual, bs.ndxSmask,
                                                         bs.sNaN, lin.p, C, Psi, SVol, bs.ELB, 1,
                                                         bs.gibbsburn, crn["uELB"], return_flags=True)
            out["elb_flags_stable"] = sflags
        shadowrate = draws[:, :, 0]
        Xn, Yn = rebuild_XY(bs, shadowrate)
        out.update(X=Xn, Y=Yn, shadowrate=shadowrate, elb_flags=flags)
    return out
