"""Oracle (CPU restatement) of the hybrid shadow-rate sampler mcmcVARhybridGibbs.m —
TEST INFRASTRUCTURE ONLY (see ccmm_oracle.py).

PARITY UNPINNED (MATLAB reference, no fixtures).  Follows the reference as
written: X = [1, lags of the shadow-rate data, Xffrlags] with Xffrlags the lags
of the actual policy rates floored at the ELB (mcmcVARhybridGibbs.m:65-90), the
Minnesota prior extended by the FFRlags block (:236-298), CTA with the chain's
single design (:376), the linear A/SV/PHI blocks (:380-418), and the ELB step
(:420-537) with companion PAI(1:Kshadow,:) and Yhatactual = Xffrlags * PAIactual.
The reference draws the shadow rates by accept-first PS proposals with
gibbsdrawShadowrates as the fallback (:458-483); the proposal sampler
VARTVPSVprecisionsamplerNaN is in the absent em-matlabbox toolbox, so the Gibbs
draw (100 burn-in + 1 passes) serves every sweep here, as in ccmm_oracle_bh.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import ccmm_oracle as O


@dataclass
class HybridSetup:
    lin: O.Setup            # Y0 (actual data), X0 = [1, lags, Xffrlags], priors (K = Kshadow + Ns p)
    Kshadow: int            # 1 + N p  (:90)
    Xffrlags: np.ndarray    # T x Ns p, floored at the ELB (:81-82)
    ndxS: np.ndarray        # shadow-rate variable indices (0-based)
    ndxSmask: np.ndarray    # bool N (elb.ndxS, :206)
    Ydata: np.ndarray       # Nobs x N, censored shadow-rate cells zeroed (:178-186)
    elbT0: int
    elbT: int
    sNaN: np.ndarray        # Ns x elbT (:210)
    X0: np.ndarray          # Kshadow: elb.X0 = X(elbT0+1, 1:Kshadow)' (:231)
    ELB: float
    gibbsburn: int = 100


def hybrid_setup(thisT, p, np_, data0, ydates0, ndxS, minnesotaPriorMean, ELBbound, elbT0,
                 doRATSprior=True, logy2offset=O.LOGY2OFFSET):
    """mcmcVARhybridGibbs.m:33-339 (thisT 1-based)."""
    base = O.var_setup(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior, logy2offset)
    theta = [0.04, 0.25, 100, 2] if doRATSprior else [0.05, 0.5, 100, 2]
    data = base.data
    Nobs, N = data.shape
    ndxS = np.asarray(ndxS)
    Ns = ndxS.size
    Kshadow = 1 + N * p
    # FFRlags(t, (l-1)Ns + s) = data(t-l, ndxS(s)), floored at the ELB (:77-82; strict '<')
    FFRlags = np.zeros((Nobs, p * Ns))
    for l in range(1, p + 1):
        FFRlags[p:, (l - 1) * Ns:l * Ns] = data[p - l:Nobs - l, :][:, ndxS]
    Xffrlags = FFRlags[p:, :].copy()
    Xffrlags[Xffrlags < ELBbound] = ELBbound
    X = np.hstack([base.X, Xffrlags])
    T, K = X.shape
    # prior of the FFRlags block (:275-291), AR_s2 from the actual data (:240-246)
    AR_s2 = np.sum(base.ARresid ** 2, axis=0) / (T - 2)
    sig = np.zeros((p * Ns, N))
    for i in range(N):
        for l in range(1, p + 1):
            for s in range(Ns):
                j = ndxS[s]
                if i == j:
                    sig[(l - 1) * Ns + s, i] = theta[0] / (l ** theta[3])
                else:
                    sig[(l - 1) * Ns + s, i] = (AR_s2[i] / AR_s2[j]) * theta[0] * theta[1] / (l ** theta[3])
    iVdiag = np.vstack([base.iVdiag, 1.0 / sig])                 # :297, 337
    iVb = np.vstack([base.iVb, np.zeros((p * Ns, N))])         # MU_pai rows of FFRlags = 0 (:276, 298)
    Xjumpoff = np.concatenate([base.Xjumpoff, np.zeros(p * Ns)])
    for l in range(1, p + 1):                                  # :117-121
        Xjumpoff[Kshadow + (l - 1) * Ns:Kshadow + l * Ns] = data[Nobs - l, ndxS]
    Xjumpoff[Kshadow:] = np.maximum(Xjumpoff[Kshadow:], ELBbound)
    lin = O.Setup(N=N, p=p, T=T, K=K, X=X, Y=base.Y, ARresid=base.ARresid, iVdiag=iVdiag,
                  iVb=iVb, sPHI=base.sPHI, dPHI=base.dPHI, Vol_0mean=base.Vol_0mean,
                  Vol_0vcvsqrt=base.Vol_0vcvsqrt, Xjumpoff=Xjumpoff, data=data,
                  logy2offset=logy2offset)
    # ELB data (:178-218)
    Smask = np.isin(np.arange(N), ndxS)
    Ydata = data.copy()
    sr = Ydata[:, ndxS].copy()
    sr[sr <= ELBbound] = np.nan
    Ydata[:, ndxS] = sr
    yNaNall = np.isnan(Ydata)
    Ydata[yNaNall] = 0.0
    yNaN = yNaNall[p:, :]
    elbT = max(0, T - elbT0)
    if elbT > 0 and np.any(yNaN[:elbT0, ndxS]):
        raise ValueError("something off about elbT0")
    sNaN = yNaN[elbT0:, :].T[Smask, :]
    X0 = X[elbT0, :Kshadow].copy() if elbT > 0 else np.zeros(Kshadow)
    return HybridSetup(lin=lin, Kshadow=Kshadow, Xffrlags=Xffrlags, ndxS=ndxS, ndxSmask=Smask,
                       Ydata=Ydata, elbT0=elbT0, elbT=elbT, sNaN=sNaN, X0=X0, ELB=ELBbound)


def hybrid_crn_sizes(hs: HybridSetup, nproposals=0):
    lin = hs.lin
    out = O.crn_sizes(lin.N, lin.K, lin.T, lin.dPHI) + [
        ("uELB", (len(hs.ndxS), hs.elbT, hs.gibbsburn + 1))]
    if nproposals:
        out.append(("zPS", (int(hs.sNaN.sum()), int(nproposals))))
    return out


def hybrid_draw_crn(rng, hs: HybridSetup, nproposals=0):
    return {name: (rng.random(shape) if name.startswith("u") else rng.standard_normal(shape))
            for name, shape in hybrid_crn_sizes(hs, nproposals)}


def ps_shadowrate(hs: HybridSetup, PAI, A, sqrtht, zPS):
    """mcmcVARhybridGibbs.m:446-483: PS proposals from the precision sampler
    (ccmm_oracle_bh.precision_sampler_nan) with PAIshadow = PAI(1:Kshadow,:) and the
    actual-rate lags' fit as intercept; returns (shadowrate or None, ndxAccept, the first proposal
    shadowrateProposals(:,:,1) = missingrate, :486)."""
    from .ccmm_oracle_bh import precision_sampler_nan
    lin = hs.lin
    N, p, Ks = lin.N, lin.p, hs.Kshadow
    _, _, SVol, Yhatactual = elb_state_space(hs, PAI, np.linalg.inv(A), sqrtht)
    PAIshadow = PAI[:Ks, :]
    pai0 = PAIshadow[0, :][:, None] + Yhatactual                                    # :448
    pai3 = PAIshadow[1:, :].T.reshape(N, N, p, order="F")                           # :449
    invbbb = A[:, :, None] / SVol[:, None, :]                                        # :450
    elbY0 = hs.X0[1:1 + N * p].reshape(N, p, order="F")
    yNaN = np.zeros((N, hs.elbT), bool)
    yNaN[hs.ndxS, :] = hs.sNaN
    Y = np.where(yNaN, 0.0, hs.Ydata[lin.p + hs.elbT0:, :].T)
    YY = precision_sampler_nan(pai3, invbbb, Y, yNaN, elbY0, pai0, zPS).reshape(N, hs.elbT, -1,
                                                                                order="F")
    props = YY[hs.ndxS, :, :]
    for k in range(props.shape[2]):                                                  # :466-471
        if np.all(props[:, :, k][hs.sNaN] < hs.ELB):
            return props[:, :, k], k + 1, props[:, :, 0]
    return None, 0, props[:, :, 0]


def elb_state_space(hs: HybridSetup, PAI, invA, sqrtht):
    """mcmcVARhybridGibbs.m:223-232, 426-441: C = elb.A, Psi = elb.B, SVol, Yhatactual."""
    lin = hs.lin
    N, p, Ks = lin.N, lin.p, hs.Kshadow
    PAIactual = PAI[Ks:, :]
    Yhatactual = (hs.Xffrlags[hs.elbT0:, :] @ PAIactual).T
    C = np.zeros((Ks, Ks))
    C[0, 0] = 1.0
    C[1 + N:, 1:1 + N * (p - 1)] = np.eye(N * (p - 1))
    C[1:1 + N, :] = PAI[:Ks, :].T
    Psi = np.zeros((Ks, N))
    Psi[1:1 + N, :] = invA
    SVol = sqrtht[hs.elbT0:, :].T
    return C, Psi, SVol, Yhatactual


def rebuild_XY(hs: HybridSetup, shadowrate):
    """mcmcVARhybridGibbs.m:457, 498, 520-528."""
    lin = hs.lin
    shadowYdata = hs.Ydata.copy()
    shadowYdata[lin.p + hs.elbT0:, hs.ndxS] = shadowrate.T
    Xl, Y = O.build_lags(shadowYdata, lin.p)
    return np.hstack([Xl, hs.Xffrlags]), Y


def hybrid_init_state(hs: HybridSetup):
    return O.init_state(hs.lin)  # :351-359 (PAI = X0\Y0 with the hybrid X0)


def hybrid_sweep(st, hs: HybridSetup, crn, elb_impl="stable", use_ps=False, cta_form="kron"):
    """One sweep of mcmcVARhybridGibbs.m:362-539 with the Gibbs ELB draw, or with use_ps the
    reference's PS proposals first (:458-483, crn["zPS"]) and the Gibbs draw as fallback.
    elb_impl as in ccmm_oracle_bh.bh_sweep ("qr", "stable" or "both")."""
    lin = hs.lin
    N, K = lin.N, lin.K
    Y, X = st["Y"], st["X"]
    if cta_form == "mirror":   # the device's large-system path in its operation order
        from . import cta_mirror
        PAI, status = cta_mirror.cta_big(Y, X, N, K, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"],
                                         crn["zPAI"])
    else:
        PAI, status = O.cta(Y, X, N, K, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"],
                            crn["zPAI"])
    RESID = Y - X @ PAI
    A, invA = O.a_step(RESID, st["sqrtht"], crn["zA"])
    logy2 = np.log((RESID @ A.T) ** 2 + lin.logy2offset)
    h, h0, shocks, kai = O.sv_ksc_corrsqrt(logy2.T, st["h"].T, st["sqrtPHI"], lin.Vol_0mean,
                                          lin.Vol_0vcvsqrt, crn["uSV"], crn["zSV"])
    h = h.T
    sqrtht = np.exp(h / 2)
    sqrtPHI, PHI = O.phi_iw(shocks.T, lin.sPHI, crn["zPHI"])
    out = dict(A=A, invA=invA, PAI=PAI, sqrtht=sqrtht, h=h, sqrtPHI=sqrtPHI, PHI=PHI,
               RESID=RESID, kai=kai.T, status=status, Y=Y, X=X)
    if hs.elbT > 0:
        C, Psi, SVol, Yhatactual = elb_state_space(hs, PAI, invA, sqrtht)
        elbY = Y[hs.elbT0:, :].T
        if use_ps:
            sr, k, first = ps_shadowrate(hs, PAI, A, sqrtht, crn["zPS"])
            out["ps_accept"] = k
            out["missingrate"] = first    # shadowrateProposals(:,:,1), mcmcVARhybridGibbs.m:486
            if k:
                Xn, Yn = rebuild_XY(hs, sr)
                out.update(X=Xn, Y=Yn, shadowrate=sr)
                return out
        if elb_impl in ("qr", "both"):
            draws = O.gibbsdraw_shadowrates(elbY, hs.X0, Yhatactual, hs.ndxSmask, hs.sNaN, lin.p,
                                            C, Psi, SVol, hs.ELB, 1, hs.gibbsburn, crn["uELB"])
            out["shadowrate_qr"] = draws[:, :, 0]
        if elb_impl in ("stable", "both"):
            from .elb_fast import gibbsdraw_shadowrates_stable
            draws = gibbsdraw_shadowrates_stable(elbY, hs.X0, Yhatactual, hs.ndxSmask, hs.sNaN,
                                                 lin.p, C, Psi, SVol, hs.ELB, 1, hs.gibbsburn,
                                                 crn["uELB"])
        shadowrate = draws[:, :, 0]
        Xn, Yn = rebuild_XY(hs, shadowrate)
        out.update(X=Xn, Y=Yn, shadowrate=shadowrate)
    return out
