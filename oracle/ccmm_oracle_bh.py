"""Oracle (CPU restatement) of the block-hybrid shadow-rate sampler
mcmcVARshadowrateBlockHybrid.m — TEST INFRASTRUCTURE ONLY (see ccmm_oracle.py).

PARITY UNPINNED (MATLAB reference, no fixtures).  Follows the reference as
written: CTAsys with per-equation designs (actual-rate X for the macro block,
shadow-rate X for the yield block), the linear A/SV/PHI blocks, then the ELB
step with gibbsdrawShadowrates (QR smoothing weights, 100 burn-in + 1 Gibbs
passes: the ``m < MCMCburnin*.5`` branch, mcmcVARshadowrateBlockHybrid.m:435-437)
or the acceptance-sampling branch (:438-466) on a restatement of the absent
em-matlabbox sampler VARTVPSVprecisionsamplerNaN (precision_sampler_nan), and
the rebuild of X, Y from the shadow draws (:501-520).
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


def bh_crn_sizes(bs: BHSetup, nproposals=0):
    """Per-sweep CRN blocks; nproposals > 0 appends the PS proposal normals
    randn(nmiss, Nproposals) (VARTVPSVprecisionsamplerNaN, :439-441)."""
    lin = bs.lin
    out = O.crn_sizes(lin.N, lin.K, lin.T, lin.dPHI) + [
        ("uELB", (len(bs.ndxS), bs.elbT, bs.gibbsburn + 1))]
    if nproposals:
        out.append(("zPS", (int(bs.sNaN.sum()), int(nproposals))))
    return out


def bh_draw_crn(rng, bs: BHSetup, nproposals=0):
    out = {}
    for name, shape in bh_crn_sizes(bs, nproposals):
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


def precision_sampler_nan(pai3, invbbb, Y, yNaN, Y0, pai0, z):
    """Missing-value draws of the VAR with time-varying volatility given the observed
    cells: the interface of em-matlabbox VARTVPSVprecisionsamplerNaN (called at
    mcmcVARshadowrateBlockHybrid.m:428,439-441,471-473,483-485; source absent, PARITY
    UNPINNED — restated as the precision-based sampler its name and arguments describe).

      model:  invbbb_t (y_t - pai0_t - sum_l pai3_l y_{t-l}) = e_t ~ N(0, I),  t = 1..T,
              y_{1-l} = Y0(:, l) (the fixed pre-window lags, :426)
      stack:  AA vec(Y) = cc + e;  split vec(Y) into missing m / observed o (yNaN):
              P = AA_m' AA_m,  b = AA_m' (cc - AA_o y_o),  P = L L' (lower Cholesky)
      draw k: y_m = L' \\ (L \\ b + z_k)   (= P^-1 b + L'^-1 z_k),  z = randn(nmiss, Ndraws)

    pai3 N x N x p (pai3(:,:,l) = Phi_l), invbbb N x N x T, Y N x T (missing cells
    ignored), yNaN N x T bool, Y0 N x p, pai0 N x T, z nmiss x Ndraws (missing cells in
    vec order: month-major, variables in index order).  Returns YYdraws N*T x Ndraws
    (observed cells copied)."""
    N, T = Y.shape
    p = pai3.shape[2]
    NT = N * T
    AA = np.zeros((NT, NT))
    cc = np.zeros(NT)
    for t in range(T):
        Bt = invbbb[:, :, t]
        r = slice(t * N, (t + 1) * N)
        AA[r, r] = Bt
        c = pai0[:, t].copy()
        for l in range(1, p + 1):
            if t - l >= 0:
                AA[r, (t - l) * N:(t - l + 1) * N] = -Bt @ pai3[:, :, l - 1]
            else:
                c += pai3[:, :, l - 1] @ Y0[:, l - t - 1]
        cc[r] = Bt @ c
    m = np.asarray(yNaN, bool).ravel(order="F")
    y = np.asarray(Y, float).ravel(order="F").copy()
    y[m] = 0.0
    Am = AA[:, m]
    P = Am.T @ Am
    b = Am.T @ (cc - AA[:, ~m] @ y[~m])
    L = np.linalg.cholesky(P)
    from scipy.linalg import solve_triangular
    ybar = solve_triangular(L, b, lower=True)
    xm = solve_triangular(L.T, ybar[:, None] + np.asarray(z, float).reshape(m.sum(), -1),
                          lower=False)
    out = np.repeat(y[:, None], xm.shape[1], axis=1)
    out[m, :] = xm
    return out


def ps_inputs(bs: BHSetup, PAI, A, sqrtht):
    """Arguments of the VARTVPSVprecisionsamplerNaN calls (mcmcVARshadowrateBlockHybrid.m:
    400-426): pai3, invbbb, elb.Y (missing cells 0), elb.yNaN, elbY0, pai0."""
    lin = bs.lin
    N, p = lin.N, lin.p
    _, _, SVol, Yhatactual = elb_state_space(bs, PAI, np.linalg.inv(A), sqrtht)
    PAIshadow = PAI.copy()
    PAIshadow[np.ix_(bs.lagmask, bs.actualrateBlock)] = 0.0
    pai0 = PAIshadow[0, :][:, None] + Yhatactual                                    # :423
    pai3 = PAIshadow[1:, :].T.reshape(N, N, p, order="F")                           # :424
    invbbb = A[:, :, None] / SVol[:, None, :]                                        # :425
    elbY0 = bs.X0[1:].reshape(N, p, order="F")                                       # :426
    yNaN = np.zeros((N, bs.elbT), bool)
    yNaN[bs.ndxS, :] = bs.sNaN
    Y = np.where(yNaN, 0.0, bs.Ydata[lin.p + bs.elbT0:, :].T)
    return pai3, invbbb, Y, yNaN, elbY0, pai0


def ps_shadowrate(bs: BHSetup, PAI, A, sqrtht, zPS):
    """Acceptance-sampling branch of the ELB step (m >= MCMCburnin/2,
    mcmcVARshadowrateBlockHybrid.m:438-460): Nproposals unconstrained draws of the
    censored cells, the first whose censored cells all lie below the ELB is accepted.
    Returns (shadowrate Ns x elbT or None, ndxAccept 1-based or 0, the first proposal
    shadowrateProposals(:,:,1), which mcmcVARshadowrate.m:435 keeps as missingrate)."""
    N = bs.lin.N
    YY = precision_sampler_nan(*ps_inputs(bs, PAI, A, sqrtht), zPS)
    YY = YY.reshape(N, bs.elbT, -1, order="F")
    props = YY[bs.ndxS, :, :]                                                        # :444
    for k in range(props.shape[2]):                                                  # :446-452
        if np.all(props[:, :, k][bs.sNaN] < bs.ELB):
            return props[:, :, k], k + 1, props[:, :, 0]
    return None, 0, props[:, :, 0]


def bh_init_state(bs: BHSetup):
    st = O.init_state(bs.lin)  # Y = Y0, X = X0 (actual data), mcmcVARshadowrateBlockHybrid.m:310-316
    return st


def bh_sweep(st, bs: BHSetup, crn, return_flags=False, elb_impl="qr", use_ps=False, cta_form="kron"):
    """One sweep of mcmcVARshadowrateBlockHybrid.m:322-523: the Gibbs ELB branch
    (m < MCMCburnin/2, :435-437), or with use_ps the acceptance-sampling branch
    (:438-466: PS proposals crn["zPS"], the first accepted, else the Gibbs draw).

    elb_impl: "qr" = gibbsdrawShadowrates as written; "stable" = the same
    conditionals in the residual form of elb_fast.gibbsdraw_shadowrates_stable
    (accurate when the shadow companion matrix is explosive, where the as-written
    Ytilde = Y - Y0 cancels catastrophically); "both" = stable, with the as-written
    draw in out["shadowrate_qr"].

    cta_form: "kron" = CTAsys.m as written; "syrk" = O.cta_sys_syrk (the same posterior in
    the weighted-SYRK form; S120-sized systems); "mirror" = the device's operation order
    (oracle/cta_mirror.cta with the per-equation designs)."""
    lin = bs.lin
    N, K, T = lin.N, lin.K, lin.T
    Y, X = st["Y"], st["X"]
    Xs = [bs.Xactual if bs.actualrateBlock[j] else X for j in range(N)]
    if cta_form == "mirror":
        from . import cta_mirror
        PAI = cta_mirror.cta(Y, Xs, N, K, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"], crn["zPAI"])
        status = 0
    elif cta_form == "kron":
        XX = np.empty((T, K, N))
        XX[:, :, bs.actualrateBlock] = bs.Xactual[:, :, None]
        XX[:, :, ~bs.actualrateBlock] = X[:, :, None]
        PAI, status = O.cta_sys(Y, XX, N, K, T, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"],
                                crn["zPAI"])
    else:
        PAI, status = O.cta_sys_syrk(Y, Xs, N, K, T, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"],
                                     crn["zPAI"])
    RESID = np.empty((T, N))
    for jj in range(N):
        RESID[:, jj] = Y[:, jj] - Xs[jj] @ PAI[:, jj]
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
        if use_ps:
            sr, k, first = ps_shadowrate(bs, PAI, A, sqrtht, crn["zPS"])
            out["ps_accept"] = k
            out["missingrate"] = first    # shadowrateProposals(:,:,1), mcmcVARshadowrate.m:435
            if k:
                Xn, Yn = rebuild_XY(bs, sr)
                out.update(X=Xn, Y=Yn, shadowrate=sr, shadowrate_qr=sr, elb_flags=None,
                           elb_flags_stable=None)
                return out
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
