"""Reference-interface mirror of the MATLAB samplers, running on libccmm.

``mcmcVAR`` keeps the signature and draw-array outputs of mcmcVAR.m:1-12
(``nargout == 4`` form: PAI_all, PHI_all, invA_all, sqrtht_all) and adds
``nchains``: B independent chains run as one device batch (the
``goVAR*`` parfor over vintages/chains becomes one GPU launch sequence).
``mcmcVARshadowrateBlockHybrid`` mirrors the block-hybrid shadow-rate sampler
(outputs 1-6).  ``CTA``/``CTAsys``/``drawTruncNormal`` mirror the L2 functions.

Every numerical step goes through ``libccmm.so``; there is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _abi
from .model import build_bh, build_hybrid, build_var, initial_state

_CTX = {}


def context(device: int = 0) -> _abi.Context:
    if device not in _CTX:
        _CTX[device] = _abi.Context(device)
    return _CTX[device]


def mcmcVAR(thisT, MCMCdraws, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior,
            ndxYIELDS=None, ELBbound=0.25, check_stationarity=0, yrealized=None, fcstNdraws=None,
            fcstNhorizons=None, rndStream=1012023, doprogress=False, *, nchains=1, device=0,
            burnin=None):
    """mcmcVAR.m (linear BVAR-SV, CTA + A + SV + PHI blocks), nargout == 4.

    rndStream: integer seed of the Philox stream (the MATLAB RandStream object
    has no device equivalent; chains c = 0..nchains-1 use counter word `chain`).
    Returns PAI_all (M x K x N), PHI_all (M x N(N+1)/2), invA_all (M x N x N),
    sqrtht_all (M x T x N), each with a trailing chain axis when nchains > 1.
    """
    if check_stationarity:
        raise NotImplementedError("check_stationarity=1 (mcmcVAR.m:221-232) is not supported; "
                                  "the reference drivers all pass 0")
    doPredictiveDensity = bool(fcstNdraws)
    if doPredictiveDensity:
        if fcstNdraws % MCMCdraws != 0:  # mcmcVAR.m:97-99
            raise ValueError("fcstNdraws must be multiple of MCMCdraws")
        if yrealized is None or ndxYIELDS is None or fcstNhorizons is None:
            raise ValueError("predictive density needs yrealized, ndxYIELDS and fcstNhorizons")
    m = build_var(thisT, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior)
    B = int(nchains)
    burn = MCMCdraws if burnin is None else int(burnin)  # MCMCburnin = MCMCdraws (mcmcVAR.m:54)
    ctx = context(device)
    ch = _abi.Chains(ctx, N=m.N, p=m.p, T=m.T, B=B, ndata=1, crn=False,
                     store_capacity=MCMCdraws, seed=int(rndStream))
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    if doPredictiveDensity:
        fc = _run_with_predictive_density(ctx, ch, m, burn, MCMCdraws, ndxYIELDS, ELBbound,
                                          yrealized, fcstNdraws, fcstNhorizons, rndStream,
                                          doprogress)
    else:
        _run_chain_set(ch, burn, MCMCdraws, doprogress)
    out = ch.get_draws()
    ch.close()
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"]]
    if doPredictiveDensity:
        res += fc
    if B == 1:
        res = [a[..., 0] for a in res]
    return tuple(res)


def _run_with_predictive_density(ctx, ch, m, burn, MCMCdraws, ndxYIELDS, ELBbound, yrealized,
                                 fcstNdraws, fcstNhorizons, seed, doprogress):
    """Kept-draw loop of mcmcVAR.m:278-381 with the predictive density of each kept
    draw on the device (ccmm_fcst), then the reshapes and means of :400-425.
    Returns fcstYdraws, fcstYhat, fcstYcensorDraws, fcstYcensorHat, fcstYshadowDraws,
    fcstYshadowHat, fcstYhatRB, fcstLogscoreDraws, fcstLogscoreELBdraws,
    fcstLogscoreXdraws, fcstLogscoreIdraws (each with a trailing chain axis)."""
    N, H, B = m.N, int(fcstNhorizons), ch.B
    Nd = fcstNdraws // MCMCdraws
    yields = np.zeros(N, bool)
    yields[np.asarray(ndxYIELDS, int)] = True
    y1 = np.asarray(yrealized, float).reshape(N, -1, order="F")[:, 0]
    Xj = np.repeat(m.Xjumpoff[:, None], B, axis=1)
    fY = np.empty((N, H, Nd, MCMCdraws, B))
    fYc = np.empty_like(fY)
    yhat = np.empty((N, H, MCMCdraws, B))
    sc = np.empty((4, Nd, MCMCdraws, B))
    _run_chain_set(ch, burn, 0, doprogress)
    for d in range(MCMCdraws):
        ch.sweep(1, store=True)
        st = ch.get_state()
        out = ctx.fcst(st["PAI"], st["invA"], st["h"][-1, :, :], st["sqrtPHI"], Xj, y1, yields,
                       ELBbound, H, Nd, seed=seed, sweep=burn + d)
        fY[:, :, :, d, :], fYc[:, :, :, d, :], yhat[:, :, d, :], sc[:, :, d, :] = out[:4]
    fYd = fY.reshape(N, H, fcstNdraws, B, order="F")
    fYcd = fYc.reshape(N, H, fcstNdraws, B, order="F")
    fYs = fYd.copy()
    sh = fYs[yields]
    sh[sh < ELBbound] = ELBbound  # :407-411
    fYs[yields] = sh
    scores = [sc[k].reshape(fcstNdraws, B, order="F") for k in range(4)]
    return [fYd, fYd.mean(axis=2), fYcd, fYcd.mean(axis=2), fYs, fYs.mean(axis=2),
            yhat.mean(axis=2)] + scores


def _run_chain_set(ch, burn, MCMCdraws, doprogress, step=50):
    done = 0
    while done < burn:
        n = min(step, burn - done)
        ch.sweep(n, store=False)
        done += n
        if doprogress:
            print(f"burn-in {done}/{burn}")
    done = 0
    while done < MCMCdraws:
        n = min(step, MCMCdraws - done)
        ch.sweep(n, store=True)
        done += n
        if doprogress:
            print(f"draws {done}/{MCMCdraws}")


def mcmcVARshadowrateBlockHybrid(thisT, MCMCdraws, p, np_, data0, ydates0, actualrateBlock,
                                 minnesotaPriorMean, doRATSprior, ndxSHADOWRATE, ndxOTHERYIELDS,
                                 doELBsampling, doELBsampleAlternate, ELBbound, elbT0,
                                 check_stationarity=0, IRF1scale=None, IRFcumcode=None,
                                 yrealized=None, fcstNdraws=None, fcstNhorizons=None,
                                 rndStream=1012023, doprogress=False, *, nchains=1, device=0,
                                 burnin=None, gibbsburn=100):
    """mcmcVARshadowrateBlockHybrid.m:1-14, outputs PAI_all, PHI_all, invA_all,
    sqrtht_all, shadowrate_all (M x Nshadowrates x elbT), missingrate_all (NaN).

    The ELB step is the Gibbs sampler of the ``m < MCMCburnin*.5`` branch
    (:435-437) at every sweep: the acceptance-sampling branch needs
    VARTVPSVprecisionsamplerNaN from the absent em-matlabbox toolbox.
    Indices are 0-based; actualrateBlock is a bool vector of length N."""
    if check_stationarity:
        raise NotImplementedError("check_stationarity=1 is not supported; the reference drivers "
                                  "all pass 0")
    if not doELBsampling or doELBsampleAlternate:
        raise NotImplementedError("doELBsampling=false / doELBsampleAlternate=true need the "
                                  "missing-data sampler VARTVPSVprecisionsamplerNaN (absent "
                                  "em-matlabbox); out of scope")
    if fcstNdraws or IRF1scale is not None:
        raise NotImplementedError("predictive density / IRF outputs are a later row (SURVEY §8f)")
    bm = build_bh(thisT, p, np_, data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS,
                  minnesotaPriorMean, ELBbound, elbT0, doRATSprior,
                  actualrateBlock=actualrateBlock)
    if bm.warn_elbT0:
        import warnings
        warnings.warn("elbT0 + 1 should be a missing obs, but it is not ...")  # :203-205
    m = bm.var
    B = int(nchains)
    burn = MCMCdraws if burnin is None else int(burnin)
    ch = _abi.Chains(context(device), N=m.N, p=m.p, T=m.T, B=B, ndata=1, crn=False,
                     store_capacity=MCMCdraws, seed=int(rndStream),
                     model=_abi.MODEL_BLOCKHYBRID, Ns=len(bm.ndxS), elbTmax=bm.elbT,
                     elb_gibbsburn=gibbsburn, elb=ELBbound)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm.ndxS, bm.actual_block)
    ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    out = ch.get_draws()
    ch.close()
    sr = out.get("shadowrate_all", np.full((MCMCdraws, len(bm.ndxS), 0, B), np.nan))
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"], sr,
           np.full((MCMCdraws, len(bm.ndxS), bm.elbT, B), np.nan)]
    if B == 1:
        res = [a[..., 0] for a in res]
    return tuple(res)


def mcmcVARhybridGibbs(thisT, MCMCdraws, p, np_, data0, ydates0, actualrateWeight,
                       minnesotaPriorMean, doRATSprior, ndxSHADOWRATE, ndxOTHERYIELDS, doELBsampling,
                       doELBsampleAlternate, ELBbound, elbT0, check_stationarity=0, IRF1scale=None,
                       IRFcumcode=None, yrealized=None, fcstNdraws=None, fcstNhorizons=None,
                       rndStream=1012023, doprogress=False, *, nchains=1, device=0, burnin=None,
                       gibbsburn=100):
    """mcmcVARhybridGibbs.m:1-14, outputs PAI_all (M x K x N, K = 1 + N p + Ns p),
    PHI_all, invA_all, sqrtht_all, shadowrate_all (M x Nshadowrates x elbT),
    missingrate_all (NaN: it is the first PS proposal, :486).

    The reference draws the shadow rates by accept-first PS proposals with the Gibbs
    sampler as fallback (:458-483); the proposal sampler VARTVPSVprecisionsamplerNaN
    is in the absent em-matlabbox toolbox, so the Gibbs draw serves every sweep.
    actualrateWeight is unused, as in the reference (:16).  Indices are 0-based."""
    if check_stationarity:
        import warnings
        warnings.warn("no stationarity check for hybrid model")  # :22-24
    if not doELBsampling or doELBsampleAlternate:
        raise NotImplementedError("doELBsampling=false / doELBsampleAlternate=true need the "
                                  "missing-data sampler VARTVPSVprecisionsamplerNaN (absent "
                                  "em-matlabbox); out of scope")
    if fcstNdraws or IRF1scale is not None:
        raise NotImplementedError("predictive density / IRF outputs are a later row (SURVEY §8f)")
    hm = build_hybrid(thisT, p, np_, data0, ydates0, ndxSHADOWRATE, minnesotaPriorMean, ELBbound,
                      elbT0, doRATSprior)
    if hm.warn_elbT0:
        import warnings
        warnings.warn("elbT0 + 1 should be a missing obs, but it is not ...")  # :216-218
    m = hm.var
    B = int(nchains)
    burn = MCMCdraws if burnin is None else int(burnin)
    ch = _abi.Chains(context(device), N=m.N, p=m.p, T=m.T, B=B, ndata=1, crn=False,
                     store_capacity=MCMCdraws, seed=int(rndStream), model=_abi.MODEL_HYBRID,
                     Ns=len(hm.ndxS), elbTmax=hm.elbT, elb_gibbsburn=gibbsburn, elb=ELBbound)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(hm.ndxS, None)
    ch.set_elb_slot(0, hm.elbT0, hm.sNaN)
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    out = ch.get_draws()
    ch.close()
    sr = out.get("shadowrate_all", np.full((MCMCdraws, len(hm.ndxS), 0, B), np.nan))
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"], sr,
           np.full((MCMCdraws, len(hm.ndxS), hm.elbT, B), np.nan)]
    if B == 1:
        res = [a[..., 0] for a in res]
    return tuple(res)


def CTA(Y, X, N, K, T, A_, sqrtht, iV, iVb_prior, PAI, rndStream=None, *, device=0):
    """CTA.m:1 signature.  iV may be the NK x NK diagonal precision or its diagonal;
    rndStream may be None (Philox) or a K x N array of standard normals (CRN)."""
    iVd = np.diag(iV) if np.ndim(iV) == 2 else np.asarray(iV)
    out, _ = context(device).cta(Y, X, np.asarray(A_)[..., None], np.asarray(sqrtht)[..., None],
                                 iVd.reshape(K, N, order="F"),
                                 np.asarray(iVb_prior).reshape(K, N, order="F"),
                                 np.asarray(PAI)[..., None],
                                 None if rndStream is None else np.asarray(rndStream)[..., None])
    return out[..., 0]


def CTAsys(Y, X, N, K, T, A_, sqrtht, iV, iVb_prior, PAI, rndStream=None, *, device=0):
    """CTAsys.m:1 signature: X is T x K x N (one design per equation)."""
    iVd = np.diag(iV) if np.ndim(iV) == 2 else np.asarray(iV)
    out, _ = context(device).cta(Y, X, np.asarray(A_)[..., None], np.asarray(sqrtht)[..., None],
                                 iVd.reshape(K, N, order="F"),
                                 np.asarray(iVb_prior).reshape(K, N, order="F"),
                                 np.asarray(PAI)[..., None],
                                 None if rndStream is None else np.asarray(rndStream)[..., None])
    return out[..., 0]


def drawTruncNormal(mu, sqrtVCV, elb, u):
    """drawTruncNormal.m:1 with the numeric-uniform form of the stream argument."""
    v, _ = _abi.draw_trunc_normal(mu, sqrtVCV, elb, u)
    return v


def _logmeanexp(x, axis=0):
    """log(mean(exp(x))) with the max shift of goVARshadowrateBlockHybrid.m:438-439."""
    x = np.asarray(x, float)
    m = np.max(x, axis=axis, keepdims=True)
    return np.squeeze(np.log(np.mean(np.exp(x - m), axis=axis, keepdims=True)) + m, axis=axis)


def realized_values(data0, thisT, fcstNhorizons, ndxSHADOWRATE, ELBbound):
    """yrealized of one vintage (goVAR.m:252-267 == goVARshadowrateBlockHybrid.m:267-283):
    the data rows after the 1-based jump-off ``thisT`` (NaN past the end of the sample),
    with the shadow-rate series floored at the ELB."""
    data0 = np.asarray(data0, float)
    Tdata, N = data0.shape
    H = int(fcstNhorizons)
    yreal = np.full((N, H), np.nan)
    nreal = max(0, min(H, Tdata - thisT))
    yreal[:, :nreal] = data0[thisT:thisT + nreal].T
    if ELBbound is not None and ndxSHADOWRATE is not None and len(ndxSHADOWRATE):
        s = np.asarray(ndxSHADOWRATE, int)
        ys = yreal[s, :]
        ys[ys < ELBbound] = ELBbound  # NaN compares false: missing months stay NaN
        yreal[s, :] = ys
    return yreal


def _rank_device(dist, device):
    """Device of this rank: explicit ``device`` wins; with a process group the rank's
    LOCAL_RANK (one process per GPU, torchrun layout); else device 0."""
    if device is not None:
        return int(device)
    if dist is not None:
        from . import distributed as dm
        return dm.world_from_env().local_rank
    return 0


def goVAR_batch(data0, ydates0, Tjumpoffs, p, np_, MCMCdraws, fcstNdraws, fcstNhorizons,
                minnesotaPriorMean, ndxYIELDS, ELBbound=0.25, doRATSprior=True, *, nchains=1,
                rndStream=1012023, dist=None, device=None, burnin=None, run_vintage=None,
                ndxSHADOWRATE=None):
    """The quasi-real-time OOS loop of goVAR.m:242 / goVARshadowrateBlockHybrid.m:258-517
    for the linear sampler: every vintage thisT in Tjumpoffs runs mcmcVAR with its
    predictive density; vintages are sharded over ranks longest-processing-time first
    (distributed.lpt_assign, no collective while sampling) and the per-vintage results
    are gathered at the end (one all-gather).

    Per vintage: fcstYmvlogscore{,X,I} = log mean exp over the fcstNdraws x nchains
    one-step log-score draws (:437-447), fcstYhat (N x H, mean over draws), and the
    censored ELB log score.  yrealized = the data rows after the jump-off (NaN past the
    end of the sample) with the ``ndxSHADOWRATE`` series floored at the ELB
    (goVAR.m:262-267; ``realized_values``).  ``run_vintage(thisT, yrealized, seed)``
    replaces the mcmcVAR call (tests use it to drive the sharding on CPU).  ``device``
    defaults to the rank's LOCAL_RANK under a process group.  Returns a dict on every rank.
    """
    from . import distributed as dm
    data0 = np.asarray(data0, float)
    Nobs, N = data0.shape
    K = N * p + 1
    rank = dist.get_rank() if dist is not None else 0
    size = dist.get_world_size() if dist is not None else 1
    device = _rank_device(dist, device)
    Tjumpoffs = [int(t) for t in Tjumpoffs]
    costs = [dm.unit_cost(t - p, K, N) for t in Tjumpoffs]
    mine = dm.lpt_assign(costs, size)[rank]
    H = int(fcstNhorizons)
    local = {}
    for v in mine:
        thisT = Tjumpoffs[v]
        yreal = realized_values(data0, thisT, H, ndxSHADOWRATE, ELBbound)
        seed = int(rndStream) + 7919 * v  # per-vintage stream (initRandStreams analogue)
        if run_vintage is not None:
            ls, lsELB, lsX, lsI, fYhat = run_vintage(thisT, yreal, seed)
        else:
            out = mcmcVAR(thisT, MCMCdraws, p, np_, data0, ydates0, minnesotaPriorMean,
                          doRATSprior, ndxYIELDS=ndxYIELDS, ELBbound=ELBbound, yrealized=yreal,
                          fcstNdraws=fcstNdraws, fcstNhorizons=H, rndStream=seed,
                          nchains=nchains, device=device, burnin=burnin)
            fYhat = out[5]
            ls, lsELB, lsX, lsI = out[11], out[12], out[13], out[14]
            if nchains > 1:
                fYhat = fYhat.mean(axis=-1)
        summ = [_logmeanexp(np.ravel(a)) for a in (ls, lsELB, lsX, lsI)]
        local[v] = np.concatenate([np.array(summ), np.ravel(fYhat, order="F")])
    allv = dm.gather_summaries(dist, local, None)
    S = np.stack([allv[v] for v in range(len(Tjumpoffs))], axis=1)
    return dict(fcstYmvlogscore=S[0], fcstYmvlogscoreELB=S[1], fcstYmvlogscoreX=S[2],
                fcstYmvlogscoreI=S[3], fcstYhat=S[4:].reshape(N, H, -1, order="F"),
                assignment=dm.lpt_assign(costs, size))
