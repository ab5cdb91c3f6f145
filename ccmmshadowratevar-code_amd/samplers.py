"""Reference-interface mirror of the MATLAB samplers, running on libccmm.

``mcmcVAR`` keeps the signature and draw-array outputs of mcmcVAR.m:1-12
(``nargout == 4`` form: PAI_all, PHI_all, invA_all, sqrtht_all) and adds
``nchains``: B independent chains run as one device batch (the
``goVAR*`` parfor over vintages/chains becomes one GPU launch sequence).
``mcmcVARshadowrateBlockHybrid`` mirrors the block-hybrid shadow-rate sampler
(outputs 1-13: draws and the predictive density).  ``goVARshadowrateBlockHybrid_batch``
is the quasi-real-time OOS run over all vintages as one device batch per GPU.  ``CTA``/``CTAsys``/``CTAsysAswitching``/``drawTruncNormal`` mirror the L2 functions.

Every numerical step goes through ``libccmm.so``; there is no CPU fallback.
"""
from __future__ import annotations

import warnings

import numpy as np

from . import _abi
from .model import build_bh, build_hybrid, build_var, elbT0_of, initial_state

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
        fc = _run_with_predictive_density(ch, m, burn, MCMCdraws, ndxYIELDS, ELBbound,
                                          yrealized, fcstNdraws, fcstNhorizons, doprogress)
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


def _run_with_predictive_density(ch, m, burn, MCMCdraws, ndxYIELDS, ELBbound, yrealized,
                                 fcstNdraws, fcstNhorizons, doprogress):
    """Kept-draw loop of mcmcVAR.m:278-381 with the predictive density of each kept draw
    simulated inside the chain set (ccmm_chains_set_fcst: no host round trip per draw),
    then the reshapes and means of :400-425.  Returns fcstYdraws, fcstYhat,
    fcstYcensorDraws, fcstYcensorHat, fcstYshadowDraws, fcstYshadowHat, fcstYhatRB,
    fcstLogscoreDraws, fcstLogscoreELBdraws, fcstLogscoreXdraws, fcstLogscoreIdraws (each
    with a trailing chain axis)."""
    N, H, B = m.N, int(fcstNhorizons), ch.B
    Nd = fcstNdraws // MCMCdraws
    yields = np.zeros(N, bool)
    yields[np.asarray(ndxYIELDS, int)] = True
    y1 = np.asarray(yrealized, float).reshape(N, -1, order="F")[:, 0]
    ch.set_fcst(H, Nd, yields, keep_paths=True)
    ch.set_fcst_slot(0, y1)
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    fc = ch.get_fcst(paths=True)
    fYd = fc["paths"].reshape(N, H, fcstNdraws, B, order="F")
    fYcd = fc["paths_censored"].reshape(N, H, fcstNdraws, B, order="F")
    fYs = fYd.copy()
    sh = fYs[yields]
    sh[sh < ELBbound] = ELBbound  # :407-411
    fYs[yields] = sh
    scores = [fc["scores"][:, :, k, :].reshape(fcstNdraws, B, order="F") for k in range(4)]
    return [fYd, fYd.mean(axis=2), fYcd, fYcd.mean(axis=2), fYs, fYs.mean(axis=2),
            fc["yhatsum"] / MCMCdraws] + scores


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
                                 burnin=None, gibbsburn=100, Nproposals=1000, elb_ps=True,
                                 stats=None):
    """mcmcVARshadowrateBlockHybrid.m:1-14, outputs PAI_all, PHI_all, invA_all,
    sqrtht_all, shadowrate_all (M x Nshadowrates x elbT), missingrate_all (NaN: the draw of the
    doELBsampleAlternate branch, off in every reference driver, :470-478).

    The ELB step follows :433-466: the Gibbs sampler for m < MCMCburnin/2, then the
    acceptance-sampling branch (Nproposals draws of the precision sampler restated from
    the absent VARTVPSVprecisionsamplerNaN, first accepted, else the Gibbs draw).
    elb_ps=False keeps the Gibbs branch at every sweep.  ``stats`` (a dict, optional)
    receives countELBaccept / countELBacceptBurnin / stackAccept (:303-305, 453-460).
    Indices are 0-based; actualrateBlock is a bool vector of length N."""
    if check_stationarity:
        raise NotImplementedError("check_stationarity=1 is not supported; the reference drivers "
                                  "all pass 0")
    if not doELBsampling or doELBsampleAlternate:
        raise NotImplementedError("doELBsampling=false / doELBsampleAlternate=true need the "
                                  "missing-data sampler VARTVPSVprecisionsamplerNaN (absent "
                                  "em-matlabbox); out of scope")
    if IRF1scale is not None:
        raise NotImplementedError("IRF outputs (doIRF1) are a later row (SURVEY §8f rank 4)")
    doPredictiveDensity = bool(fcstNdraws)
    if doPredictiveDensity:
        if fcstNdraws % MCMCdraws != 0:  # :123-126
            raise ValueError("fcstNdraws must be multiple of MCMCdraws")
        if yrealized is None or fcstNhorizons is None:
            raise ValueError("predictive density needs yrealized and fcstNhorizons")
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
    if elb_ps and Nproposals:
        ch.set_elb_ps(Nproposals, max(1, -(-burn // 2)))  # m >= MCMCburnin * .5 (:435)
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    if doPredictiveDensity:
        N, H = m.N, int(fcstNhorizons)
        Nd = fcstNdraws // MCMCdraws
        ndxYIELDS = np.union1d(bm.ndxS, bm.ndxO)                  # :83
        yields = np.zeros(N, bool)
        yields[ndxYIELDS] = True
        ch.set_fcst(H, Nd, yields, keep_paths=True)
        ch.set_fcst_slot(0, np.asarray(yrealized, float).reshape(N, -1, order="F")[:, 0])
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    if doPredictiveDensity:
        fc = ch.get_fcst(paths=True)
    if stats is not None and elb_ps and Nproposals:
        ps = ch.get_ps()
        stats.update(countELBaccept=ps["countAccept"], countELBacceptBurnin=ps["countAcceptBurnin"],
                     stackAccept=ps["stackAccept"])
    out = ch.get_draws()
    ch.close()
    sr = out.get("shadowrate_all", np.full((MCMCdraws, len(bm.ndxS), 0, B), np.nan))
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"], sr,
           np.full((MCMCdraws, len(bm.ndxS), bm.elbT, B), np.nan)]
    if doPredictiveDensity:
        # outputs 7-13 (:692-748): censored draws / mean, uncensored yields (shadow-rate
        # forecasts) / mean, the three one-step score draws
        fYd = fc["paths_censored"].reshape(N, H, fcstNdraws, B, order="F")
        fSd = fc["paths"][yields].reshape(int(yields.sum()), H, fcstNdraws, B, order="F")
        sc = [fc["scores"][:, :, k, :].reshape(fcstNdraws, B, order="F") for k in (1, 2, 3)]
        res += [fYd, fYd.mean(axis=2), fSd, fSd.mean(axis=2), sc[0], sc[1], sc[2]]
    if B == 1:
        res = [a[..., 0] for a in res]
    return tuple(res)


def mcmcVARshadowrate(thisT, MCMCdraws, p, np_, data0, ydates0, minnesotaPriorMean, doRATSprior,
                      doPAIactual, ndxSHADOWRATE, ndxOTHERYIELDS, doELBsampling, ELBbound, elbT0,
                      check_stationarity=0, IRF1scale=None, IRFcumcode=None, yrealized=None,
                      fcstNdraws=None, fcstNhorizons=None, rndStream=1012023, doprogress=False, *,
                      nchains=1, device=0, burnin=None, gibbsburn=100, Nproposals=100, stats=None):
    """mcmcVARshadowrate.m:1-17 (the shadow-rate VAR without the actual-rate block): CTA on
    the shadow-rate design for every equation (:322-326), the ELB step of the block hybrid
    with YHAT0 = [] (Gibbs for m < MCMCburnin/2, then elb.Nproposals = 100 PS proposals,
    :397-436), and the linear model's predictive density whose censored recursion floors
    ndxOTHERYIELDS only (:539-546), chain set model CCMM_MODEL_SHADOWRATE.  Outputs 1-17:
    PAI_all, PHI_all, invA_all, sqrtht_all, shadowrate_all, missingrate_all (proposal 1 of the
    sweep's PS draws, :435, 498; NaN for Gibbs sweeps), fcstYdraws, fcstYhat, fcstYcensorDraws, fcstYcensorHat, fcstShadowrateDraws, fcstShadowrateHat,
    fcstYhatRB, fcstLogscoreDraws, fcstLogscoreXdraws, fcstLogscoreIdraws, stackAccept
    (:630-700).  Indices 0-based."""
    if check_stationarity:
        raise NotImplementedError("check_stationarity=1 is not supported; the reference drivers "
                                  "all pass 0")
    if doPAIactual:
        raise NotImplementedError("doPAIactual = true (CTA on the actual data, :322-324) is not built")
    if not doELBsampling:
        raise NotImplementedError("doELBsampling = false (missing-data treatment) is not built")
    if IRF1scale is not None:
        raise NotImplementedError("in-sampler IRF outputs: use samplers.generateGIRF")
    doPredictiveDensity = bool(fcstNdraws)
    if doPredictiveDensity and fcstNdraws % MCMCdraws:
        raise ValueError("fcstNdraws must be multiple of MCMCdraws")
    N = np.asarray(data0).shape[1]
    bm = build_bh(thisT, p, np_, data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean,
                  ELBbound, elbT0, doRATSprior, actualrateBlock=np.zeros(N, bool))
    m = bm.var
    B = int(nchains)
    burn = MCMCdraws if burnin is None else int(burnin)
    ch = _abi.Chains(context(device), N=m.N, p=m.p, T=m.T, B=B, ndata=1, crn=False,
                     store_capacity=MCMCdraws, seed=int(rndStream), model=_abi.MODEL_SHADOWRATE,
                     Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=gibbsburn, elb=ELBbound)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm.ndxS, None)
    ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
    if Nproposals:
        ch.set_elb_ps(Nproposals, max(1, -(-burn // 2)))      # m >= MCMCburnin * .5 (:403)
        ch.keep_missingrate(True)                             # missingrate = proposal 1 (:435, 498)
    ndxY = np.union1d(bm.ndxS, bm.ndxO)
    yields = np.zeros(N, bool)
    yields[ndxY] = True
    if doPredictiveDensity:
        H, Nd = int(fcstNhorizons), fcstNdraws // MCMCdraws
        ch.set_fcst(H, Nd, yields, keep_paths=True)
        other = np.zeros(N, bool)
        other[bm.ndxO] = True
        ch.set_fcst_censor(other)                             # :539-546
        ch.set_fcst_slot(0, np.asarray(yrealized, float).reshape(N, -1, order="F")[:, 0])
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    stack = np.zeros((MCMCdraws, B), np.int32)
    if Nproposals:
        ps = ch.get_ps()
        stack = ps["stackAccept"]
        if stats is not None:
            stats.update(countELBaccept=ps["countAccept"], countELBacceptBurnin=ps["countAcceptBurnin"])
    fc = ch.get_fcst(paths=True) if doPredictiveDensity else None
    miss = ch.get_missingrate() if Nproposals and bm.elbT else None
    out = ch.get_draws()
    ch.close()
    sr = out.get("shadowrate_all", np.full((MCMCdraws, len(bm.ndxS), 0, B), np.nan))
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"], sr,
           miss[:, :, :bm.elbT] if miss is not None else np.full_like(sr, np.nan)]
    if doPredictiveDensity:
        fYd = fc["paths"].reshape(N, H, fcstNdraws, B, order="F").copy()
        fSd = fYd[ndxY].copy()                                # fcstShadowrateDraws (:640)
        yd = fYd[ndxY]
        yd[yd < ELBbound] = ELBbound                          # :642-645
        fYd[ndxY] = yd
        fYc = fc["paths_censored"].reshape(N, H, fcstNdraws, B, order="F").copy()
        yc = fYc[bm.ndxS]
        yc[yc < ELBbound] = ELBbound                          # :676-681
        fYc[bm.ndxS] = yc
        RB = fc["yhatsum"] / MCMCdraws                        # :639
        fYhat = RB.copy()
        fYhat[ndxY] = fYd[ndxY].mean(axis=2)                  # :683-684
        sc = [fc["scores"][:, :, k, :].reshape(fcstNdraws, B, order="F") for k in (1, 2, 3)]
        res += [fYd, fYhat, fYc, fYc.mean(axis=2), fSd, RB[ndxY], RB, sc[0], sc[1], sc[2]]
    res.append(stack)
    if B == 1:
        res = [a[..., 0] for a in res]
    return tuple(res)


def mcmcVARhybridGibbs(thisT, MCMCdraws, p, np_, data0, ydates0, actualrateWeight,
                       minnesotaPriorMean, doRATSprior, ndxSHADOWRATE, ndxOTHERYIELDS, doELBsampling,
                       doELBsampleAlternate, ELBbound, elbT0, check_stationarity=0, IRF1scale=None,
                       IRFcumcode=None, yrealized=None, fcstNdraws=None, fcstNhorizons=None,
                       rndStream=1012023, doprogress=False, *, nchains=1, device=0, burnin=None,
                       gibbsburn=100, Nproposals=1000, elb_ps=True, stats=None):
    """mcmcVARhybridGibbs.m:1-14, outputs PAI_all (M x K x N, K = 1 + N p + Ns p),
    PHI_all, invA_all, sqrtht_all, shadowrate_all (M x Nshadowrates x elbT),
    missingrate_all (proposal 1 of each sweep's PS draws, :486; NaN with elb_ps=False); with
    fcstNdraws the predictive
    density of every kept draw simulated on the device (:566-635) and outputs 7-13 (:703-751):
    fcstYdraws (yields floored at the ELB), fcstYhat, fcstShadowrateDraws, fcstShadowrateHat,
    fcstLogscoreDraws, fcstLogscoreXdraws, fcstLogscoreIdraws.

    The shadow rates are drawn by accept-first PS proposals at every sweep with the Gibbs
    sampler as fallback (:458-483), the proposal sampler restated from the absent
    em-matlabbox VARTVPSVprecisionsamplerNaN (elb_ps=False: Gibbs every sweep).
    actualrateWeight is unused, as in the reference (:16).  Indices are 0-based."""
    if check_stationarity:
        import warnings
        warnings.warn("no stationarity check for hybrid model")  # :22-24
    if not doELBsampling or doELBsampleAlternate:
        raise NotImplementedError("doELBsampling=false / doELBsampleAlternate=true need the "
                                  "missing-data sampler VARTVPSVprecisionsamplerNaN (absent "
                                  "em-matlabbox); out of scope")
    if IRF1scale is not None:
        raise NotImplementedError("in-sampler IRF outputs: use samplers.generateGIRF(hybrid=True)")
    doPredictiveDensity = bool(fcstNdraws)
    if doPredictiveDensity:
        if fcstNdraws % MCMCdraws:
            raise ValueError("fcstNdraws must be multiple of MCMCdraws")
        if yrealized is None or fcstNhorizons is None:
            raise ValueError("predictive density needs yrealized and fcstNhorizons")
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
    if elb_ps and Nproposals:
        ch.set_elb_ps(Nproposals, 1)                   # every sweep (:458)
        ch.keep_missingrate(True)                      # missingrate = proposal 1 (:486)
    N = m.N
    ndxYIELDS = np.union1d(hm.ndxS, np.asarray(ndxOTHERYIELDS, int))
    if doPredictiveDensity:
        H, Nd = int(fcstNhorizons), fcstNdraws // MCMCdraws
        yields = np.zeros(N, bool)
        yields[ndxYIELDS] = True
        ch.set_fcst(H, Nd, yields, keep_paths=True)
        ch.set_fcst_slot(0, np.asarray(yrealized, float).reshape(N, -1, order="F")[:, 0])
    st = initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    _run_chain_set(ch, burn, MCMCdraws, doprogress)
    if stats is not None and elb_ps and Nproposals:
        ps = ch.get_ps()
        stats.update(countELBaccept=ps["countAccept"] + ps["countAcceptBurnin"],
                     stackAccept=ps["stackAccept"])
    fc = ch.get_fcst(paths=True) if doPredictiveDensity else None
    miss = ch.get_missingrate() if elb_ps and Nproposals and hm.elbT else None
    out = ch.get_draws()
    ch.close()
    sr = out.get("shadowrate_all", np.full((MCMCdraws, len(hm.ndxS), 0, B), np.nan))
    res = [out["PAI_all"], out["PHI_all"], out["invA_all"], out["sqrtht_all"], sr,
           miss[:, :, :hm.elbT] if miss is not None else np.full((MCMCdraws, len(hm.ndxS), hm.elbT, B), np.nan)]
    if doPredictiveDensity:
        fYu = fc["paths"].reshape(N, H, fcstNdraws, B, order="F")          # uncensored simulation
        fSd = fYu[ndxYIELDS].copy()                                         # fcstShadowrateDraws (:704)
        fYd = fc["paths_censored"].reshape(N, H, fcstNdraws, B, order="F")  # yields floored (:707-711)
        sc = [fc["scores"][:, :, k, :].reshape(fcstNdraws, B, order="F") for k in (1, 2, 3)]
        res += [fYd, fYd.mean(axis=2), fSd, fSd.mean(axis=2), sc[0], sc[1], sc[2]]
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


def CTAsysAswitching(Y, X, N, K, T, A_, Aelb_, atELB, sqrtht, iV, iVb_prior, PAI, rndStream=None, *, device=0):
    """CTAsysAswitching.m:1 signature (the Aelb model's coefficient block): X is T x K x N, the
    months with atELB true use Aelb_ instead of A_ (CTAsysAswitching.m:61-80)."""
    iVd = np.diag(iV) if np.ndim(iV) == 2 else np.asarray(iV)
    out, _ = context(device).cta_aswitching(Y, X, np.asarray(A_)[..., None], np.asarray(Aelb_)[..., None],
                                            atELB, np.asarray(sqrtht)[..., None],
                                            iVd.reshape(K, N, order="F"),
                                            np.asarray(iVb_prior).reshape(K, N, order="F"),
                                            np.asarray(PAI)[..., None],
                                            None if rndStream is None else np.asarray(rndStream)[..., None])
    return out[..., 0]


def gibbsdrawShadowratesB3(Y, STATE0, ndxS, sNaN, p, A, B, SVol, elbBound, Ndraws=1, burnin=0, rndStream=None,
                           *, device=0):
    """gibbsdrawShadowratesB3.m:1 signature (12 arguments): Y Ny x T, STATE0 K, ndxS logical Ny, sNaN
    Ns x T, A K x K, B K x Ny or K x Ny x T (month-varying, :49-51), SVol Ny x T; rndStream: the
    uniforms rand(Ns, T, burnin + Ndraws) (:163) or None (Philox).  Returns Ns x T x Ndraws."""
    B = np.asarray(B, float)
    u = None if rndStream is None else np.asarray(rndStream, float)[..., None]
    out = context(device).gibbs_shadowrates_b3(np.asarray(Y, float)[..., None], np.asarray(STATE0, float)[:, None],
                                               ndxS, sNaN, p, np.asarray(A, float)[..., None], B[..., None],
                                               np.asarray(SVol, float)[..., None], elbBound, burnin=burnin,
                                               u=u, Ndraws=Ndraws, month_varying=B.ndim == 3)
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


# ---------------------------------------------------------------------------------------
# Block-hybrid quasi-real-time OOS batch (goVARshadowrateBlockHybrid.m) on the device

def datenum(y, m, d):
    """MATLAB datenum of a calendar date (proleptic Gregorian, day 1 = 0000-01-01)."""
    import datetime
    return float(datetime.date(y, m, d).toordinal() + 366)


def _normcdf(x):
    import math
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


# goVARshadowrateBlockHybrid.m:141
SET_QUANTILES = np.array([.5, 2.5, 5, _normcdf(-1) * 100, 25, 75, (1 - _normcdf(-1)) * 100, 95, 97.5,
                          99.5])


def max_var_roots(PAI_all, N, p, threads=16):
    """max(abs(eig(comp))) of every draw's companion matrix (goVARshadowrateBlockHybrid.m:
    384-392), PAI_all M x K x N; host LAPACK (dgeev) over a thread pool."""
    from concurrent.futures import ThreadPoolExecutor
    M = PAI_all.shape[0]
    Np = N * p

    def one(P):
        comp = np.zeros((Np, Np))
        comp[N:, :Np - N] = np.eye(Np - N)
        comp[:N, :] = P[1:1 + Np, :].T
        return float(np.max(np.abs(np.linalg.eigvals(comp))))

    with ThreadPoolExecutor(max_workers=threads) as ex:
        return np.array(list(ex.map(one, [PAI_all[m] for m in range(M)])))


def save_qrt_mat(filename, res, *, data, ydates, p, ncode, tcode, cumcode, ndxSHADOWRATE,
                 ndxOTHERYIELDS, ELBbound, actualrateBlock, datalabel, modellabel, MCMCdraws,
                 fcstNhorizons, doQuarterly=False):
    """The QRT summary file of goVARshadowrateBlockHybrid.m:641-669 (varlist: data, ydates, p,
    Tjumpoffs, N, ncode, tcode, cumcode, fcst*, fcstNhorizons, PAI*, shadowrate*, missingrate*,
    ndx*, ELBbound, ELBdummy, actualrateBlock, datalabel, modellabel, doQuarterly,
    setQuantiles, MCMCdraws) from a goVARshadowrateBlockHybrid_batch result.  MATLAB
    -v7.3 is HDF5; this writes the same names and shapes as a v5 MAT-file (scipy.io.savemat).
    Index variables are 1-based as in MATLAB; missingrate* are NaN (doELBsampleAlternate is
    false in the driver)."""
    from scipy.io import savemat
    data = np.asarray(data, float)
    ndxS1 = np.asarray(ndxSHADOWRATE, int) + 1
    ndxO1 = np.asarray(ndxOTHERYIELDS, int) + 1
    Tdata = data.shape[0]
    Ns = ndxS1.size
    V = len(res["Tjumpoffs"])
    m = dict(data=data, ydates=np.asarray(ydates, float)[:, None], p=float(p),
             Tjumpoffs=np.asarray(res["Tjumpoffs"], float)[:, None], N=float(data.shape[1]),
             ncode=np.array(list(ncode), dtype=object)[None, :], tcode=np.asarray(tcode, float)[None, :],
             cumcode=np.asarray(cumcode, bool)[None, :], fcstNhorizons=float(fcstNhorizons),
             ndxSHADOWRATE=ndxS1.astype(float)[None, :], ndxOTHERYIELDS=ndxO1.astype(float)[None, :],
             ndxYIELDS=np.union1d(ndxS1, ndxO1).astype(float)[None, :], ELBbound=float(ELBbound),
             ELBdummy=data[:, ndxS1 - 1] <= ELBbound,
             actualrateBlock=np.asarray(actualrateBlock, bool)[None, :], datalabel=datalabel,
             modellabel=modellabel, doQuarterly=bool(doQuarterly), MCMCdraws=float(MCMCdraws),
             setQuantiles=np.asarray(res.get("setQuantiles", SET_QUANTILES), float)[None, :],
             missingrateVintagesMid=np.full((Tdata, Ns, V), np.nan),
             missingrateVintagesTails=np.full((Tdata, Ns, 4, V), np.nan))
    for k, v in res.items():
        # the reference's wildcards; shadowratePSRFchains (psrf across chains) is not a reference output
        if k.startswith(("fcst", "PAI", "shadowrate")) and k != "shadowratePSRFchains" and isinstance(v, np.ndarray):
            m[k] = v[None, :] if v.ndim == 1 else v
    savemat(filename, m, do_compression=True)
    return sorted(m)


def matlab_prctile(x, pct, axis=0):
    """MATLAB prctile (Statistics Toolbox): NaN values removed, the n sorted values sit at
    percentiles 100 (i - 0.5) / n, linear interpolation between, clamped outside = numpy 'hazen'
    (NaN where every value is NaN)."""
    x = np.asarray(x, float)
    if not np.isnan(x).any():
        return np.percentile(x, pct, axis=axis, method="hazen")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)                # all-NaN slices: NaN
        return np.nanpercentile(x, pct, axis=axis, method="hazen")


def _bh_units(data0, ydates0, Tjumpoffs, p, np_, ndxSHADOWRATE, ndxOTHERYIELDS,
              minnesotaPriorMean, ELBbound, elbT0, doRATSprior, fcstNhorizons, model="blockhybrid"):
    """Host setup of every vintage (mcmcVARshadowrateBlockHybrid.m:30-295; model="hybrid":
    mcmcVARhybridGibbs.m:33-339; model="shadowrate": mcmcVARshadowrate.m, every equation on the
    shadow-rate design) and its yrealized (goVARshadowrateBlockHybrid.m:267-283)."""
    out = []
    N = np.asarray(data0).shape[1]
    for thisT in Tjumpoffs:
        if model == "hybrid":
            bm = build_hybrid(int(thisT), p, np_, data0, ydates0, ndxSHADOWRATE, minnesotaPriorMean,
                              ELBbound, elbT0, doRATSprior)
        else:
            bm = build_bh(int(thisT), p, np_, data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS,
                          minnesotaPriorMean, ELBbound, elbT0, doRATSprior,
                          **({"actualrateBlock": np.zeros(N, bool)} if model == "shadowrate" else {}))
        yr = realized_values(data0, int(thisT), fcstNhorizons, ndxSHADOWRATE, ELBbound)
        out.append((int(thisT), bm, yr))
    return out


def _bh_chain_set(ctx, units, C, *, seed, ids, store_capacity, gibbsburn, ELBbound, ndxYIELDS,
                  fcstNhorizons=None, Nd=None, keep_paths=False, model="blockhybrid"):
    """One device-resident chain set holding every unit (vintage) as a data slot with C
    chains each (the parfor over vintages as one batch), reference initialisation per
    chain (:308-317), predictive density on every stored sweep."""
    bm0 = units[0][1]
    N, p = bm0.var.N, bm0.var.p
    Tmax = max(u[1].var.T for u in units)
    elbTmax = max(max(u[1].elbT for u in units), 1)
    B = C * len(units)
    hybrid = model == "hybrid"
    shadow = model == "shadowrate"
    ch = _abi.Chains(ctx, N=N, p=p, T=Tmax, B=B, ndata=len(units), crn=False,
                     store_capacity=store_capacity, seed=int(seed),
                     model=_abi.MODEL_HYBRID if hybrid else (_abi.MODEL_SHADOWRATE if shadow else _abi.MODEL_BLOCKHYBRID),
                     Ns=len(bm0.ndxS), elbTmax=elbTmax, elb_gibbsburn=gibbsburn, elb=ELBbound)
    for s, (_, bm, _) in enumerate(units):
        m = bm.var
        ch.set_data(s, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm0.ndxS, None if (hybrid or shadow) else bm0.actual_block)
    yields = np.zeros(N, bool)
    yields[np.asarray(ndxYIELDS, int)] = True
    if fcstNhorizons:
        ch.set_fcst(fcstNhorizons, Nd, yields, keep_paths=keep_paths)
        if shadow:                                   # mcmcVARshadowrate.m:539-546: ndxOTHERYIELDS only
            other = yields.copy()
            other[np.asarray(bm0.ndxS, int)] = False
            ch.set_fcst_censor(other)
    slots = np.repeat(np.arange(len(units)), C).astype(np.int32)
    ch.set_slots(slots)
    K = bm0.var.K
    init = dict(PAI=np.zeros((K, N, B), order="F"), A=np.zeros((N, N, B), order="F"),
                sqrtht=np.ones((Tmax, N, B), order="F"), h=np.zeros((Tmax, N, B), order="F"),
                sqrtPHI=np.zeros((N, N, B), order="F"))
    for s, (_, bm, yr) in enumerate(units):
        ch.set_elb_slot(s, bm.elbT0, bm.sNaN)
        if fcstNhorizons:
            ch.set_fcst_slot(s, yr[:, 0])
        st = initial_state(bm.var, C)
        T = bm.var.T
        for k in init:
            if k in ("sqrtht", "h"):
                init[k][:T, :, s * C:(s + 1) * C] = st[k]
            else:
                init[k][..., s * C:(s + 1) * C] = st[k]
    ch.set_state(init["PAI"], init["A"], init["sqrtht"], init["h"], init["sqrtPHI"])
    ch.set_rng_ids(ids)
    return ch, slots, yields


def goVARshadowrateBlockHybrid_batch(data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS,
                                     minnesotaPriorMean, *, Tjumpoffs=None, p=12, np_=12,
                                     MCMCdraws=1000, fcstNdraws=None, fcstNhorizons=48,
                                     ELBbound=0.25, doRATSprior=True, nchains=1, burnin=None,
                                     gibbsburn=100, rndStream=1012023, dist=None, device=None,
                                     chunk=50, max_retries=2, keep_draws=False, progress=False,
                                     Nproposals=1000, elb_ps=True, postprocess=False, cumcode=None,
                                     setQuantiles=None, maxlambda=False, model="blockhybrid",
                                     engine="python"):
    """The quasi-real-time OOS run of goVARshadowrateBlockHybrid.m:126-517 for the block-
    hybrid shadow-rate VAR, as ONE device-resident chain set per rank: every vintage
    thisT in Tjumpoffs (default: ydates > 2008-12, :127) is a data slot of the set with
    ``nchains`` chains (the parfor over vintages, :258, becomes the batch), vintages are
    sharded over ranks longest-processing-time first (all chains of a vintage on one
    rank), and nothing crosses ranks until the end (one all-gather of the per-vintage
    summaries).

    Per chain: MCMCdraws burn-in + MCMCdraws kept sweeps (mcmcVARshadowrateBlockHybrid.m:
    56-58); every kept sweep stores the draw and simulates fcstNdraws / MCMCdraws forecast
    paths on the device (:550-625).  The ELB step is the Gibbs sampler for m < MCMCburnin/2
    and the accept-first PS proposals (Nproposals) after, as mcmcVARshadowrateBlockHybrid.m:
    433-466 (elb_ps=False: Gibbs every sweep).  Philox streams are keyed by the global unit
    (vintage index * nchains + chain), so results do not depend on the number of ranks.

    Failure recovery (:287-310): chains whose blocks flagged a non-SPD pivot
    (ccmm_chains_get_status) have their vintage re-run from scratch on fresh streams, up
    to ``max_retries`` times.

    Returns (every rank) a dict with, per vintage v: fcstYmvlogscore{,X,I} (log mean exp
    of the fcstNdraws * nchains one-step score draws, :437-447), fcstYhat (N x H x V,
    censored paths), fcstShadowYhat (Nyields x H x V), fcstYrealized, fcstYhaterror,
    PAImean / PAIstdev (K x N x V, :376-378), shadowrateVintagesMid / Tails
    (Tdata x Ns (x 4) x V, median and prctile [5 25 75 95] of the kept shadow rates,
    :331-334,497-506), plus run statistics.

    postprocess=True adds the per-vintage post-processing of :349-480 on the device
    (ccmm_chains_summaries; every kept draw and forecast path of the set stays in HBM):
    fcstYmedian / fcstYmederror / fcstYcrps / fcstYquantiles (N x H (x Nq) x V), their
    cumulated forms fcstYcum* (cumsum over horizons for ``cumcode``), fcstShadowYmedian /
    fcstShadowYquantiles, PAImedian / PAIquantiles, the score draws fcstYmvlogscore*Draws;
    setQuantiles default goVARshadowrateBlockHybrid.m:141.  maxlambda=True adds
    drawsMaxVARroot (max |eig| of each draw's companion matrix, :382-392, host LAPACK).

    model="hybrid" runs goVARhybrid.m instead (goVARhybrid_batch): mcmcVARhybridGibbs per
    vintage (K = N p + 1 + Ns p, PS proposals at every sweep, :458), modellabel ELBhybrid; the
    max-root block is commented out in that driver (:383-430), so maxlambda is refused.

    model="shadowrate" runs goVARshadowrate.m (goVARshadowrate_batch): mcmcVARshadowrate per
    vintage (every equation on the shadow-rate design, elb.Nproposals = 100).  Its forecast
    outputs follow that driver: fcstYhat is the Rao-Blackwellised mean with the yields replaced by
    the mean of their ELB-floored draws (mcmcVARshadowrate.m:639-645, 683-684), fcstYhatRB the
    Rao-Blackwellised mean, fcstShadowYhat its yield rows, fcstYcensorhat the mean of the censored
    paths (other yields floored inside the simulation, shadow rates after, :539-546, 676-681),
    missingrateVintagesMid / Tails the median and prctile [5 25 75 95] of the kept missingrate_all
    (goVARshadowrate.m:345-348, 523-529); postprocess=True adds the ydraws / ycumdraws /
    ycensordraws summaries of goVARshadowrate.m:356-495 (fcstYcensor{median,crps,quantiles}), all
    on the device (ccmm_chains_summaries_floor).  The forecast paths of every vintage stay in HBM
    until the summaries are taken (Python engine only).

    keep_draws=True also returns the kept draws per vintage: PAI_all[v] (M x K x N x C) and
    shadowrate_all[v] (M x Ns x elbT x C).  shadowratePSRF (Ns x V) is DiagnosticsShadowrate of each
    vintage's kept shadow rates over the months at the ELB (:322-325, ccmm_shadowrate_psrf: the
    reference's first-third / last-third split of each chain, averaged over the C chains);
    shadowratePSRFchains the psrf across the C chains (NaN for one chain; not a reference output).

    engine="native" runs the rank's vintage loop (chain set, burn-in, kept sweeps, forecast
    records, device summaries, retries) inside the library, ccmm_run_batch (include/ccmm.h): the
    same Philox streams and the same per-vintage results (keep_draws / maxlambda not available
    there)."""
    import time
    from . import distributed as dm
    data0 = np.asarray(data0, float)
    ydates0 = np.asarray(ydates0, float)
    Tdata, N = data0.shape
    ndxSHADOWRATE = np.asarray(ndxSHADOWRATE, int)
    ndxOTHERYIELDS = np.asarray(ndxOTHERYIELDS, int)
    ndxYIELDS = np.union1d(ndxSHADOWRATE, ndxOTHERYIELDS)
    if Tjumpoffs is None:
        Tjumpoffs = np.flatnonzero(ydates0 > datenum(2008, 12, 1)) + 1   # 1-based (:127)
    Tjumpoffs = [int(t) for t in Tjumpoffs]
    if fcstNdraws is None:
        fcstNdraws = 10 * MCMCdraws                                      # :38
    if fcstNdraws % MCMCdraws:
        raise ValueError("fcstNdraws must be multiple of MCMCdraws")     # :123-126
    Nd = fcstNdraws // MCMCdraws
    burn = MCMCdraws if burnin is None else int(burnin)
    C = int(nchains)
    H = int(fcstNhorizons)
    # ELB window start, global over vintages (:131-134)
    elbT0 = elbT0_of(data0, ndxSHADOWRATE, ELBbound, p)
    startELB = elbT0 + 1 + p                                            # 1-based month
    rank = dist.get_rank() if dist is not None else 0
    size = dist.get_world_size() if dist is not None else 1
    device = _rank_device(dist, device)
    hybrid = model == "hybrid"
    is_sr = model == "shadowrate"
    if model not in ("blockhybrid", "hybrid", "shadowrate"):
        raise ValueError(f"unknown model {model!r}")
    if is_sr and engine == "native":
        raise ValueError("model='shadowrate' runs on the Python engine (ccmm_chains_summaries_floor)")
    smask = np.zeros(N, bool)
    smask[ndxSHADOWRATE] = True
    elbdummy = data0[:, ndxSHADOWRATE] <= ELBbound                      # ELBdummy, :131
    if hybrid and maxlambda:
        raise ValueError("goVARhybrid.m computes no max VAR roots (:383-430 commented out)")
    K = N * p + 1 + (ndxSHADOWRATE.size * p if hybrid else 0)
    costs = [dm.unit_cost(t - p, K, N, n_cens=dm.censored_months(data0, ndxSHADOWRATE, ELBbound, startELB, t)) * C
             for t in Tjumpoffs]
    assignment = dm.lpt_assign(costs, size)
    mine = assignment[rank]
    t0 = time.perf_counter()
    units = _bh_units(data0, ydates0, [Tjumpoffs[v] for v in mine], p, np_, ndxSHADOWRATE,
                      ndxOTHERYIELDS, minnesotaPriorMean, ELBbound, elbT0, doRATSprior, H,
                      model=model) if mine else []
    t_setup = time.perf_counter() - t0
    ctx = context(device)
    Ns = ndxSHADOWRATE.size
    chunk = max(1, min(int(chunk), MCMCdraws))

    cumcode = None if cumcode is None else np.asarray(cumcode, bool)
    pct = np.asarray(SET_QUANTILES if setQuantiles is None else setQuantiles, float)

    def run(vidx, attempt):
        """Run the vintages vidx (indices into `mine`); returns per-vintage results and
        the list of vintages whose chains were flagged."""
        us = [units[i] for i in vidx]
        ids = np.array([(mine[i] * C + c) + attempt * 1_000_003 for i in vidx for c in range(C)],
                       dtype=np.uint32)
        # postprocess (and the shadow-rate VAR, whose yhat needs the floored draws): every kept
        # draw and forecast path stays on the device until the per-vintage summaries
        # (ccmm_chains_summaries) have been taken
        dev = postprocess or is_sr
        ch, slots, yields = _bh_chain_set(ctx, us, C, seed=rndStream, ids=ids,
                                          store_capacity=MCMCdraws if dev else chunk,
                                          gibbsburn=gibbsburn, ELBbound=ELBbound,
                                          ndxYIELDS=ndxYIELDS, fcstNhorizons=H, Nd=Nd,
                                          keep_paths=dev, model=model)
        use_ps = bool(elb_ps and Nproposals and ch.elbTmax)
        if use_ps:
            # block hybrid, shadow rate: m >= MCMCburnin * .5 (:435, mcmcVARshadowrate.m:403);
            # hybrid: every sweep (mcmcVARhybridGibbs.m:458)
            ch.set_elb_ps(Nproposals, 1 if hybrid else max(1, -(-burn // 2)))
            if is_sr:
                ch.keep_missingrate(True)                  # mcmcVARshadowrate.m:435, 498
        B = ch.B
        done = 0
        while done < burn:
            n = min(chunk, burn - done)
            ch.sweep(n, store=False)
            done += n
            if progress:
                print(f"[rank {rank}] burn-in {done}/{burn} ({time.perf_counter() - t1:.1f} s)", flush=True)
        scores = np.empty((Nd, MCMCdraws, 4, B))
        fYsum = np.zeros((N, H, B))
        fYcsum = np.zeros((N, H, B))
        yhsum = np.zeros((N, H, B))
        Psum = np.zeros((K, N, B))
        P2sum = np.zeros((K, N, B))
        elbTmax = ch.elbTmax
        shadow = np.empty((MCMCdraws, Ns, elbTmax, B)) if elbTmax else None
        PAIdraws = np.empty((MCMCdraws, K, N, B)) if (keep_draws or maxlambda) else None
        post = {}
        done = 0
        while done < MCMCdraws:
            n = min(chunk, MCMCdraws - done)
            ch.sweep(n, store=True)
            if not dev:
                fc = ch.get_fcst()
                dr = ch.get_draws(which={"PAI_all", "shadowrate_all"})
                scores[:, done:done + n] = fc["scores"]
                fYsum += fc["fYsum"]
                fYcsum += fc["fYcsum"]
                P = dr["PAI_all"]
                Psum += P.sum(axis=0)
                P2sum += (P * P).sum(axis=0)
                if shadow is not None:
                    shadow[done:done + n] = dr["shadowrate_all"]
                if PAIdraws is not None:
                    PAIdraws[done:done + n] = P
            done += n
            if progress:
                print(f"[rank {rank}] kept {done}/{MCMCdraws} ({time.perf_counter() - t1:.1f} s)", flush=True)
        miss = None
        if dev:
            # goVARshadowrateBlockHybrid.m:349-480 on the device, per vintage (data slot)
            for k, i in enumerate(vidx):
                thisT, bm, yr = units[i]
                ycr = np.array(yr, float)
                if cumcode is not None:
                    ycr[cumcode] = np.cumsum(ycr[cumcode], axis=1)              # :353
                if is_sr:
                    # goVARshadowrate.m:356-495: ydraws = uncensored paths, yields floored; the
                    # censored paths with the shadow rates floored; shadowratedraws unfloored
                    q = dict(ycr=ycr, pa=ch.summaries(2, k, pct=pct if postprocess else ()))
                    q["yd"] = ch.summaries(0, k, realized=yr if postprocess else None,
                                           pct=pct if postprocess else (), floor_rows=yields, floor=ELBbound)
                    q["yz"] = ch.summaries(1, k, realized=yr if postprocess else None,
                                           pct=pct if postprocess else (), floor_rows=smask, floor=ELBbound)
                    if postprocess:
                        q["yc"] = ch.summaries(0, k, cumcode=cumcode, realized=ycr, pct=pct, floor_rows=yields,
                                               floor=ELBbound)
                        q["sh"] = ch.summaries(0, k, rows=yields, pct=pct)
                    post[i] = q
                    continue
                yd = ch.summaries(1, k, realized=yr, pct=pct)                   # ydraws
                yc = ch.summaries(1, k, cumcode=cumcode, realized=ycr, pct=pct)  # ycumdraws
                sh = ch.summaries(0, k, rows=yields, pct=pct)                   # shadowratedraws
                pa = ch.summaries(2, k, pct=pct)                                # PAI_all
                post[i] = dict(yd=yd, yc=yc, sh=sh, pa=pa, ycr=ycr)
                if progress and (k % 8 == 7 or k == len(vidx) - 1):
                    print(f"[rank {rank}] device summaries {k + 1}/{len(vidx)} vintages "
                          f"({time.perf_counter() - t1:.1f} s)", flush=True)
            fc = ch.get_fcst()
            scores[:] = fc["scores"]
            fYsum[:] = fc["fYsum"]
            fYcsum[:] = fc["fYcsum"]
            yhsum[:] = fc["yhatsum"]
            if is_sr and use_ps:
                miss = ch.get_missingrate()                                     # M x Ns x elbTmax x B
            dr = ch.get_draws(which={"shadowrate_all"} | ({"PAI_all"} if PAIdraws is not None else set()))
            if shadow is not None:
                shadow[:] = dr["shadowrate_all"]
            if PAIdraws is not None:
                PAIdraws[:] = dr["PAI_all"]
        status = ch.get_status()
        nacc = None
        if use_ps:
            psd = ch.get_ps()
            nacc = psd["countAccept"] + psd["countAcceptBurnin"]
        ch.close()
        res, failed = {}, []
        Ny = int(np.count_nonzero(yields))
        for k, i in enumerate(vidx):
            cs = slice(k * C, (k + 1) * C)
            if np.any(status[cs] & ~_abi.STATUS_INFO):  # bits 1, 64: informational (valid draws)
                failed.append(i)
                continue
            thisT, bm, yr = units[i]
            nk = MCMCdraws * C
            r = dict(thisT=thisT, yrealized=yr,
                     countELBaccept=None if nacc is None else int(nacc[cs].sum()),
                     logscore=_logmeanexp(scores[:, :, 1, cs].ravel()),
                     logscoreX=_logmeanexp(scores[:, :, 2, cs].ravel()),
                     logscoreI=_logmeanexp(scores[:, :, 3, cs].ravel()),
                     fcstYhat=fYcsum[:, :, cs].sum(axis=2) / (nk * Nd),
                     fcstShadowYhat=fYsum[ndxYIELDS][:, :, cs].sum(axis=2) / (nk * Nd))
            if is_sr:
                q = post[i]
                RB = yhsum[:, :, cs].sum(axis=2) / nk                          # mcmcVARshadowrate.m:639
                yh = RB.copy()
                yh[ndxYIELDS] = q["yd"]["mean"].reshape(N, H, order="F")[ndxYIELDS]   # :683-684
                r.update(fcstYhat=yh, fcstYhatRB=RB, fcstShadowYhat=RB[ndxYIELDS],
                         fcstYcensorhat=q["yz"]["mean"].reshape(N, H, order="F"),
                         PAImean=q["pa"]["mean"].reshape(K, N, order="F"),
                         PAIstdev=q["pa"]["stdev"].reshape(K, N, order="F"))
                if postprocess:
                    nq = pct.size
                    yc = yh.copy()
                    if cumcode is not None:
                        yc[cumcode] = np.cumsum(yc[cumcode], axis=1)
                    r.update(PAImedian=q["pa"]["median"].reshape(K, N, order="F"),
                             PAIquantiles=q["pa"]["quantiles"].reshape(K, N, nq, order="F"),
                             fcstYmedian=q["yd"]["median"].reshape(N, H, order="F"),
                             fcstYcrps=q["yd"]["crps"].reshape(N, H, order="F"),
                             fcstYquantiles=q["yd"]["quantiles"].reshape(N, H, nq, order="F"),
                             fcstYcumrealized=q["ycr"], fcstYcumhat=yc,
                             fcstYcummedian=q["yc"]["median"].reshape(N, H, order="F"),
                             fcstYcumcrps=q["yc"]["crps"].reshape(N, H, order="F"),
                             fcstYcumquantiles=q["yc"]["quantiles"].reshape(N, H, nq, order="F"),
                             fcstYcensormedian=q["yz"]["median"].reshape(N, H, order="F"),
                             fcstYcensorcrps=q["yz"]["crps"].reshape(N, H, order="F"),
                             fcstYcensorquantiles=q["yz"]["quantiles"].reshape(N, H, nq, order="F"),
                             fcstShadowYmedian=q["sh"]["median"].reshape(Ny, H, order="F"),
                             fcstShadowYquantiles=q["sh"]["quantiles"].reshape(Ny, H, nq, order="F"),
                             fcstYmvlogscoreDraws=scores[:, :, 1, cs].ravel(order="F"),
                             fcstYmvlogscoreXdraws=scores[:, :, 2, cs].ravel(order="F"),
                             fcstYmvlogscoreIdraws=scores[:, :, 3, cs].ravel(order="F"))
                if miss is not None and bm.elbT > 0:
                    # missingrate_all permuted to (Nobs, Ns, draws): MATLAB median (NaN if any draw
                    # is NaN) and prctile (NaN draws removed), goVARshadowrate.m:345-348
                    mr = miss[:, :, :bm.elbT, cs].transpose(2, 1, 0, 3).reshape(bm.elbT, Ns, -1)
                    r["missingrateMid"] = np.median(mr, axis=2)
                    r["missingrateTails"] = np.moveaxis(matlab_prctile(mr, [5, 25, 75, 95], axis=2), 0, 2)
            elif i in post:
                q = post[i]
                nq = pct.size
                r["PAImean"] = q["pa"]["mean"].reshape(K, N, order="F")
                r["PAIstdev"] = q["pa"]["stdev"].reshape(K, N, order="F")
                r["PAImedian"] = q["pa"]["median"].reshape(K, N, order="F")
                r["PAIquantiles"] = q["pa"]["quantiles"].reshape(K, N, nq, order="F")
                r["fcstYmedian"] = q["yd"]["median"].reshape(N, H, order="F")
                r["fcstYcrps"] = q["yd"]["crps"].reshape(N, H, order="F")
                r["fcstYquantiles"] = q["yd"]["quantiles"].reshape(N, H, nq, order="F")
                yh = r["fcstYhat"].copy()
                if cumcode is not None:
                    yh[cumcode] = np.cumsum(yh[cumcode], axis=1)                # :355
                r["fcstYcumrealized"] = q["ycr"]
                r["fcstYcumhat"] = yh
                r["fcstYcummedian"] = q["yc"]["median"].reshape(N, H, order="F")
                r["fcstYcumcrps"] = q["yc"]["crps"].reshape(N, H, order="F")
                r["fcstYcumquantiles"] = q["yc"]["quantiles"].reshape(N, H, nq, order="F")
                r["fcstShadowYmedian"] = q["sh"]["median"].reshape(Ny, H, order="F")
                r["fcstShadowYquantiles"] = q["sh"]["quantiles"].reshape(Ny, H, nq, order="F")
                r["fcstYmvlogscoreDraws"] = scores[:, :, 1, cs].ravel(order="F")
                r["fcstYmvlogscoreXdraws"] = scores[:, :, 2, cs].ravel(order="F")
                r["fcstYmvlogscoreIdraws"] = scores[:, :, 3, cs].ravel(order="F")
            else:
                r["PAImean"] = Psum[:, :, cs].sum(axis=2) / nk
                var = P2sum[:, :, cs].sum(axis=2) / nk - r["PAImean"] ** 2
                r["PAIstdev"] = np.sqrt(np.maximum(var, 0.0))               # std(.,1,1): 1/n
            if shadow is not None and keep_draws:
                r["shadowrate_all"] = shadow[:, :, :bm.elbT, cs].copy()     # M x Ns x elbT x C
            if shadow is not None:
                # goVARshadowrateBlockHybrid.m:322-325: DiagnosticsShadowrate per shadow rate over
                # its months at the ELB, ELBdummy(startELB:thisT, s)
                r["shadowratePSRF"] = _abi.shadowrate_psrf(shadow[..., cs], elbdummy[startELB - 1:thisT].T)
                r["shadowratePSRFchains"] = _abi.shadowrate_psrf(shadow[..., cs], elbdummy[startELB - 1:thisT].T,
                                                                 chains=True)
            if shadow is not None and bm.elbT > 0:
                # shadowrate_all permuted to (Nobs, Ns, draws) (:329-334)
                sr = shadow[:, :, :bm.elbT, cs].transpose(2, 1, 0, 3).reshape(bm.elbT, Ns, -1)
                r["shadowrateMid"] = np.median(sr, axis=2)
                r["shadowrateTails"] = np.moveaxis(matlab_prctile(sr, [5, 25, 75, 95], axis=2), 0, 2)
            if PAIdraws is not None:
                P = PAIdraws[..., cs]
                if keep_draws:
                    r["PAI_all"] = P
                if maxlambda:
                    r["drawsMaxVARroot"] = max_var_roots(np.moveaxis(P, 3, 1).reshape(-1, K, N), N, p)
            res[mine[i]] = r
            if progress and (k % 4 == 3 or k == len(vidx) - 1):
                print(f"[rank {rank}] results {k + 1}/{len(vidx)} vintages ({time.perf_counter() - t1:.1f} s)",
                      flush=True)
        return res, failed

    t1 = time.perf_counter()
    local, retries = {}, []
    todo = list(range(len(mine)))
    attempt = 0
    if engine == "native":
        if keep_draws or maxlambda:
            raise ValueError("engine='native' keeps no PAI draws (keep_draws / maxlambda)")
        local, retries = _native_batch(ctx, units, mine, C=C, N=N, p=p, K=K, Ns=Ns, H=H, Nd=Nd,
                                       MCMCdraws=MCMCdraws, burn=burn, gibbsburn=gibbsburn,
                                       Nproposals=Nproposals if elb_ps else 0, ELBbound=ELBbound,
                                       rndStream=rndStream, chunk=chunk, max_retries=max_retries,
                                       postprocess=postprocess, pct=pct, cumcode=cumcode,
                                       ndxYIELDS=ndxYIELDS, hybrid=hybrid)
        todo = []
    elif engine != "python":
        raise ValueError(f"engine must be 'python' or 'native', not {engine!r}")
    while todo:
        res, failed = run(todo, attempt)
        local.update(res)
        if failed:
            retries.append([mine[i] for i in failed])
        if not failed or attempt >= max_retries:
            todo = []
            for i in failed:                       # give up: NaN summaries for the unit
                local[mine[i]] = None
        else:
            todo = failed
        attempt += 1
    ctx.synchronize()
    t_run = time.perf_counter() - t1
    # ---- end of run: one all-gather of the per-vintage summaries
    allv = dict(local)
    if dist is not None:
        objs = [None] * size
        dist.all_gather_object(objs, local)
        for d_ in objs:
            allv.update(d_)
    V = len(Tjumpoffs)
    Ny = ndxYIELDS.size
    out = dict(Tjumpoffs=np.array(Tjumpoffs), assignment=assignment,
               fcstYmvlogscore=np.full(V, np.nan), fcstYmvlogscoreX=np.full(V, np.nan),
               fcstYmvlogscoreI=np.full(V, np.nan), fcstYhat=np.full((N, H, V), np.nan),
               fcstShadowYhat=np.full((Ny, H, V), np.nan), fcstYrealized=np.full((N, H, V), np.nan),
               PAImean=np.full((K, N, V), np.nan), PAIstdev=np.full((K, N, V), np.nan),
               countELBaccept=np.full(V, -1),
               shadowratePSRF=np.full((Ns, V), np.nan),                      # :213
               shadowratePSRFchains=np.full((Ns, V), np.nan),                # psrf across chains (no ref.)
               shadowrateVintagesMid=np.full((Tdata, Ns, V), np.nan),
               shadowrateVintagesTails=np.full((Tdata, Ns, 4, V), np.nan))
    if is_sr:
        out.update(fcstYhatRB=np.full((N, H, V), np.nan), fcstYcensorhat=np.full((N, H, V), np.nan),
                   missingrateVintagesMid=np.full((Tdata, Ns, V), np.nan),
                   missingrateVintagesTails=np.full((Tdata, Ns, 4, V), np.nan))
    if keep_draws:
        out["PAI_all"] = {}
        out["shadowrate_all"] = {}
    nq = pct.size
    if postprocess:
        for nm, shp in (("fcstYmedian", (N, H)), ("fcstYcrps", (N, H)), ("fcstYquantiles", (N, H, nq)),
                        ("fcstYcumrealized", (N, H)), ("fcstYcumhat", (N, H)), ("fcstYcummedian", (N, H)),
                        ("fcstYcumcrps", (N, H)), ("fcstYcumquantiles", (N, H, nq)),
                        ("fcstShadowYmedian", (Ny, H)), ("fcstShadowYquantiles", (Ny, H, nq)),
                        ("PAImedian", (K, N)), ("PAIquantiles", (K, N, nq)),
                        ("fcstYmvlogscoreDraws", (fcstNdraws * C,)),
                        ("fcstYmvlogscoreXdraws", (fcstNdraws * C,)),
                        ("fcstYmvlogscoreIdraws", (fcstNdraws * C,))):
            out[nm] = np.full(shp + (V,), np.nan)
        if is_sr:
            for nm, shp in (("fcstYcensormedian", (N, H)), ("fcstYcensorcrps", (N, H)),
                            ("fcstYcensorquantiles", (N, H, nq))):
                out[nm] = np.full(shp + (V,), np.nan)
    if maxlambda:
        out["drawsMaxVARroot"] = np.full((MCMCdraws * C, V), np.nan)
    jumpoff = p + elbT0                                                  # :497
    for v in range(V):
        r = allv.get(v)
        if r is None:
            continue
        out["fcstYmvlogscore"][v] = r["logscore"]
        out["fcstYmvlogscoreX"][v] = r["logscoreX"]
        out["fcstYmvlogscoreI"][v] = r["logscoreI"]
        out["fcstYhat"][..., v] = r["fcstYhat"]
        out["fcstShadowYhat"][..., v] = r["fcstShadowYhat"]
        out["fcstYrealized"][..., v] = r["yrealized"]
        out["PAImean"][..., v] = r["PAImean"]
        out["PAIstdev"][..., v] = r["PAIstdev"]
        if r.get("countELBaccept") is not None:
            out["countELBaccept"][v] = r["countELBaccept"]
        if "shadowratePSRF" in r:
            out["shadowratePSRF"][:, v] = r["shadowratePSRF"]
        if "shadowratePSRFchains" in r:
            out["shadowratePSRFchains"][:, v] = r["shadowratePSRFchains"]
        if "shadowrateMid" in r:
            thisT = r["thisT"]
            out["shadowrateVintagesMid"][jumpoff:thisT, :, v] = r["shadowrateMid"]
            out["shadowrateVintagesTails"][jumpoff:thisT, :, :, v] = r["shadowrateTails"]
        if "missingrateMid" in r:
            out["missingrateVintagesMid"][jumpoff:r["thisT"], :, v] = r["missingrateMid"]       # :523-529
            out["missingrateVintagesTails"][jumpoff:r["thisT"], :, :, v] = r["missingrateTails"]
        if keep_draws and "PAI_all" in r:
            out["PAI_all"][v] = r["PAI_all"]
        if keep_draws and "shadowrate_all" in r:
            out["shadowrate_all"][v] = r["shadowrate_all"]
        for nm in ("fcstYmedian", "fcstYcrps", "fcstYquantiles", "fcstYcumrealized", "fcstYcumhat",
                   "fcstYcummedian", "fcstYcumcrps", "fcstYcumquantiles", "fcstShadowYmedian",
                   "fcstShadowYquantiles", "PAImedian", "PAIquantiles", "fcstYmvlogscoreDraws",
                   "fcstYmvlogscoreXdraws", "fcstYmvlogscoreIdraws", "drawsMaxVARroot", "fcstYhatRB",
                   "fcstYcensorhat", "fcstYcensormedian", "fcstYcensorcrps", "fcstYcensorquantiles"):
            if nm in r and nm in out:
                out[nm][..., v] = r[nm]
    out["fcstYhaterror"] = out["fcstYrealized"] - out["fcstYhat"]                      # :453
    if is_sr:
        out["fcstYcensorhaterror"] = out["fcstYrealized"] - out["fcstYcensorhat"]      # goVARshadowrate.m:487
        if postprocess:
            out["fcstYcensormederror"] = out["fcstYrealized"] - out["fcstYcensormedian"]  # :488
    if postprocess:
        out["fcstYmederror"] = out["fcstYrealized"] - out["fcstYmedian"]              # :454
        out["fcstYcumhaterror"] = out["fcstYcumrealized"] - out["fcstYcumhat"]        # :463
        out["fcstYcummederror"] = out["fcstYcumrealized"] - out["fcstYcummedian"]     # :464
        out["setQuantiles"] = pct
    n_units = len(mine) * C
    out["stats"] = dict(rank=rank, world=size, device=device, vintages_local=len(mine),
                        units_local=n_units, sweeps_local=n_units * (burn + MCMCdraws),
                        setup_s=t_setup, run_s=t_run, retries=retries)
    return out


def _native_batch(ctx, units, mine, *, C, N, p, K, Ns, H, Nd, MCMCdraws, burn, gibbsburn, Nproposals,
                  ELBbound, rndStream, chunk, max_retries, postprocess, pct, cumcode, ndxYIELDS, hybrid):
    """The rank's vintage loop through ccmm_run_batch; returns the per-vintage result dicts of
    goVARshadowrateBlockHybrid_batch (keyed by global vintage index) and the retried vintages."""
    if not units:
        return {}, []
    yields = np.zeros(N, bool)
    yields[np.asarray(ndxYIELDS, int)] = True
    vins = []
    for i, (thisT, bm, yr) in enumerate(units):
        m = bm.var
        st = initial_state(m, 1)
        vins.append(dict(T=m.T, Y=m.Y, X=m.X, iVdiag=m.iVdiag, iVb=m.iVb, sPHI=m.sPHI, h0mean=m.Vol_0mean,
                         h0vcvsqrt=m.Vol_0vcvsqrt, PAI0=st["PAI"][..., 0], sqrtht0=st["sqrtht"][..., 0], h0init=st["h"][..., 0],
                         elbT0=bm.elbT0, sNaN=bm.sNaN, yrealized=yr, unit=mine[i]))
    bm0 = units[0][1]
    out = ctx.run_batch(model=_abi.MODEL_HYBRID if hybrid else _abi.MODEL_BLOCKHYBRID, N=N, p=p, Ns=Ns,
                        ndxS=bm0.ndxS, actual_block=None if hybrid else bm0.actual_block, ndxYields=yields,
                        nchains=C, MCMCdraws=MCMCdraws, burnin=burn, gibbsburn=gibbsburn, Nproposals=Nproposals,
                        fcstNdraws=Nd * MCMCdraws, H=H, elb=ELBbound, seed=int(rndStream), chunk=chunk,
                        max_retries=max_retries, postprocess=postprocess, pct=pct, cumcode=cumcode,
                        vintages=vins)
    res, retries = {}, []
    nq = pct.size
    Ny = int(np.count_nonzero(yields))
    for i, (thisT, bm, yr) in enumerate(units):
        a = int(out["attempts"][i])
        # one list per retry attempt, as the Python engine reports them: vintage i was retried on
        # attempts 1 .. a - 1 (a - 1 > max_retries: it failed every time)
        for k in range(1, min(a, max_retries + 2)):
            while len(retries) < k:
                retries.append([])
            retries[k - 1].append(mine[i])
        if a > max_retries + 1:
            res[mine[i]] = None
            continue
        r = dict(thisT=thisT, yrealized=yr,
                 countELBaccept=None if Nproposals == 0 else int(out["countELBaccept"][i]),
                 logscore=out["logscore"][1, i], logscoreX=out["logscore"][2, i], logscoreI=out["logscore"][3, i],
                 fcstYhat=out["fcstYhat"][..., i].copy(), fcstShadowYhat=out["fcstShadowYhat"][yields][..., i].copy(),
                 PAImean=out["PAImean"][..., i].copy(), PAIstdev=out["PAIstdev"][..., i].copy())
        if postprocess:
            ycr = np.array(yr, float)
            yh = r["fcstYhat"].copy()
            if cumcode is not None:
                ycr[cumcode] = np.cumsum(ycr[cumcode], axis=1)
                yh[cumcode] = np.cumsum(yh[cumcode], axis=1)
            r.update(PAImedian=out["PAImedian"][..., i], PAIquantiles=out["PAIquantiles"][..., i],
                     fcstYmedian=out["fcstYmedian"][..., i], fcstYcrps=out["fcstYcrps"][..., i],
                     fcstYquantiles=out["fcstYquantiles"][..., i], fcstYcumrealized=ycr, fcstYcumhat=yh,
                     fcstYcummedian=out["fcstYcummedian"][..., i], fcstYcumcrps=out["fcstYcumcrps"][..., i],
                     fcstYcumquantiles=out["fcstYcumquantiles"][..., i],
                     fcstShadowYmedian=out["fcstShadowYmedian"][..., i].reshape(Ny, H),
                     fcstShadowYquantiles=out["fcstShadowYquantiles"][..., i].reshape(Ny, H, nq),
                     fcstYmvlogscoreDraws=out["scoreDraws"][:, 1, i], fcstYmvlogscoreXdraws=out["scoreDraws"][:, 2, i],
                     fcstYmvlogscoreIdraws=out["scoreDraws"][:, 3, i])
        r["shadowratePSRF"] = out["shadowratePSRF"][:, i].copy()          # :322-325
        r["shadowratePSRFchains"] = out["shadowratePSRFchains"][:, i].copy()
        if bm.elbT > 0:
            sh = out["shadowrate_all"][:, :, :bm.elbT, :, i]                 # M x Ns x elbT x C
            sr = sh.transpose(2, 1, 0, 3).reshape(bm.elbT, Ns, -1)
            r["shadowrateMid"] = np.median(sr, axis=2)
            r["shadowrateTails"] = np.moveaxis(matlab_prctile(sr, [5, 25, 75, 95], axis=2), 0, 2)
        res[mine[i]] = r
    return res, retries


def goVARshadowrate_batch(data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean, *,
                          Nproposals=100, **kw):
    """goVARshadowrate.m (the quasi-real-time OOS run of the shadow-rate VAR, mcmcVARshadowrate per
    vintage, parfor at :265, elb.Nproposals = 100 at mcmcVARshadowrate.m:169, modellabel
    ELBsampling) as one device-resident chain set per rank; arguments and outputs of
    goVARshadowrateBlockHybrid_batch plus fcstYhatRB, fcstYcensor*, missingrateVintages*."""
    return goVARshadowrateBlockHybrid_batch(data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean,
                                            model="shadowrate", Nproposals=Nproposals, **kw)


def goVARhybrid_batch(data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean, **kw):
    """goVARhybrid.m (the quasi-real-time OOS run of the hybrid shadow-rate VAR,
    mcmcVARhybridGibbs per vintage, parfor at :258) as one device-resident chain set per rank;
    same arguments and outputs as goVARshadowrateBlockHybrid_batch (PAI* over K = N p + 1 + Ns p)."""
    return goVARshadowrateBlockHybrid_batch(data0, ydates0, ndxSHADOWRATE, ndxOTHERYIELDS, minnesotaPriorMean,
                                            model="hybrid", **kw)


# ---------------------------------------------------------------------------------------
# Generalized impulse responses (generateGIRF2linear.m / generateGIRF2blockhybrid.m)

def _ivech(v, N):
    """ivech of PHI_all's vech (PHI_((tril(PHI_))~=0), column-major lower triangle)."""
    M = np.zeros((N, N))
    r, c = np.nonzero(np.tril(np.ones((N, N))).T)   # column-major order of the lower triangle
    M[c, r] = v
    return np.tril(M) + np.tril(M, -1).T


def generateGIRF(data, ydates, irfDate, PAI_all, invA_all, PHI_all, sqrtht_all, *, p=12, np_=12,
                 cumcode=None, shock11=1.0, irfNdraws=1000, irfHorizon=120, blockhybrid=False,
                 ndxSHADOWRATE=None, ndxOTHERYIELDS=None, ELBbound=0.25, shadowrate_all=None,
                 elbT0=None, seed=1012023, device=0, hybrid=False):
    """The GIRF simulation of generateGIRF2linear.m / generateGIRF2blockhybrid.m:176-283 /
    generateGIRF2hybrid.m:168-275 (hybrid=True: PAI_all M x (K + Ns p) x N, the actual-rate
    lags of the Ns shadow-rate variables in the state, simVARhybrid) for
    one irfDate and shock scale (shock11 = IRF1scale * shocksize) over the M kept draws,
    on the device (ccmm_girf): returns fcstYhat / fcstYhat1plus / fcstYhat1minus (medians over
    the draws of the simulated mean paths), IRF1plus / IRF1minus (medians of +shock - base and
    -shock - base) with their prc70 tails (normcdf([-1 1]) * 100), and the draws themselves.
    PAI_all M x K x N, invA_all M x N x N, PHI_all M x N(N+1)/2, sqrtht_all M x T x N (VAR rows
    p+1..), shadowrate_all M x Ns x elbT (block hybrid); indices 0-based."""
    data = np.asarray(data, float)
    ydates = np.asarray(ydates, float)
    M, Kx, N = PAI_all.shape
    K = 1 + N * p
    t0 = int(np.flatnonzero(ydates == irfDate)[0])               # ndxIRFT0 - 1 (0-based)
    cum = np.zeros(N, bool) if cumcode is None else np.asarray(cumcode, bool)
    shadow = None
    if hybrid:                                                    # generateGIRF2hybrid.m:64-75
        yields = np.zeros(N, bool)
        yields[np.union1d(ndxSHADOWRATE, ndxOTHERYIELDS)] = True
        yidx = np.asarray(ndxSHADOWRATE, int)                     # the actual-rate ring
        shadow = np.zeros(N, bool)
        shadow[yidx] = True
        actual = None
        ns = K + yidx.size * p
        if Kx != ns:
            raise ValueError("hybrid PAI_all must have K + Nshadowrates p rows")
        blockhybrid_ring = True
    elif blockhybrid:
        yidx = np.union1d(ndxSHADOWRATE, ndxOTHERYIELDS)
        yields = np.zeros(N, bool)
        yields[yidx] = True
        actual = ~yields
        ns = K + yidx.size * p
        blockhybrid_ring = True
    else:
        yields = actual = None
        ns = K
        blockhybrid_ring = False
    Xj = np.zeros((ns, M))
    for mm in range(M):
        thisData = data[:t0 + 1].copy()                           # jumpoffData (:198-201)
        if blockhybrid_ring and shadowrate_all is not None and t0 + 1 - elbT0 - p > 0:
            n = t0 + 1 - elbT0 - p                                # (:166-172, 207-209)
            thisData[p + elbT0:t0 + 1, ndxSHADOWRATE] = shadowrate_all[mm, :, :n].T
        Xj[0, mm] = 1.0
        for l in range(p):
            Xj[1 + l * N:1 + (l + 1) * N, mm] = thisData[t0 - l, :N]
            if blockhybrid_ring:                                  # (:215-218; hybrid :211-214)
                Xj[K + l * yidx.size:K + (l + 1) * yidx.size, mm] = thisData[t0 - l, yidx]
    SV0 = np.asarray(sqrtht_all, float)[:, t0 - p, :].T          # SVjumpoffDraws (:164)
    sqrtPHI = np.stack([np.linalg.cholesky(_ivech(PHI_all[m], N)) for m in range(M)], -1)
    out = context(device).girf(np.moveaxis(PAI_all, 0, -1), np.moveaxis(invA_all, 0, -1), sqrtPHI, SV0,
                               Xj, irfHorizon, irfNdraws, shock11, bh=blockhybrid, actual=actual,
                               ndxYields=yields, elb=ELBbound, cumcode=cum, np_=np_, seed=seed,
                               hybrid=hybrid, ndxShadow=shadow, p=p)
    base, plus, minus = out[:, :, 0, :], out[:, :, 1, :], out[:, :, 2, :]
    prc70 = np.array([_normcdf(-1), _normcdf(1)]) * 100
    ctx = context(device)

    def med_tails(d):          # median / prctile over the draws (dimension 3)
        s = ctx.draw_summaries(d.reshape(N * irfHorizon, M).T, pct=prc70)
        return s["median"].reshape(N, irfHorizon), s["quantiles"].reshape(N, irfHorizon, 2)

    res = dict(fcstYHATdraws=base, fcstYHATdraws1plus=plus, fcstYHATdraws1minus=minus)
    res["fcstYhat"] = med_tails(base)[0]
    res["fcstYhat1plus"] = med_tails(plus)[0]
    res["fcstYhat1minus"] = med_tails(minus)[0]
    res["IRF1plus"], res["IRF1plusTails"] = med_tails(plus - base)       # :268-276
    res["IRF1minus"], res["IRF1minusTails"] = med_tails(minus - base)
    return res
