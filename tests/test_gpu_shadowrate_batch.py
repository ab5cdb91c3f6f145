"""goVARshadowrate.m's vintage loop (samplers.goVARshadowrate_batch: mcmcVARshadowrate per vintage as
one device-resident chain set, the per-vintage summaries of goVARshadowrate.m:329-529 on the device
through ccmm_chains_summaries_floor).

One vintage with nchains chains draws from the same Philox streams (unit 0, chains 0..C-1) as the
single-vintage wrapper samplers.mcmcVARshadowrate (itself CRN-checked against the oracle in
test_gpu_shadowrate.py), so the batch's summaries must equal numpy summaries of the wrapper's
outputs 1-17 (fcstYdraws with the yields floored, fcstYcensorDraws, fcstShadowrateDraws,
fcstYhatRB, missingrate_all, PAI_all) to summation order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ELB = 0.25


def _crps(y, x):
    """crpsDraws (the declared estimator of ccmm_post.hip): mean|x - y| - sum_i (2i - n - 1) x_(i) / n^2."""
    xs = np.sort(x, axis=-1)
    n = xs.shape[-1]
    w = 2.0 * np.arange(1, n + 1) - n - 1.0
    return np.mean(np.abs(xs - y[..., None]), axis=-1) - (xs @ w) / (n * n)


def _close(name, got, want, tol=1e-12):
    got, want = np.asarray(got, float), np.asarray(want, float)
    assert got.shape == want.shape, (name, got.shape, want.shape)
    assert np.array_equal(np.isnan(got), np.isnan(want)), name
    m = ~np.isnan(want)
    err = float(np.max(np.abs(got[m] - want[m]) / np.maximum(np.abs(want[m]), 1.0))) if m.any() else 0.0
    print(f"  {name}: max rel {err:.2e}")
    assert err < tol, (name, err)


def test_shadowrate_batch_matches_single_vintage_sampler(pkg, fred):
    S = pkg.samplers
    d = fred
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], ELB)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    e0 = pkg.model.elbT0_of(d["data"], ndxS, ELB, 12)
    N = d["data"].shape[1]
    thisT = len(d["ydates"]) - 24
    H, M, Nd, C, burn = 12, 6, 2, 2, 4
    yreal = S.realized_values(d["data"], thisT, H, ndxS, ELB)
    one = S.mcmcVARshadowrate(thisT, M, 12, 12, d["data"], d["ydates"], mpm, True, False, ndxS, ndxO, True, ELB, e0,
                              yrealized=yreal, fcstNdraws=M * Nd, fcstNhorizons=H, burnin=burn, gibbsburn=5,
                              nchains=C)
    PAI, _, _, _, sr, miss, fYd, _, fYc, _, fSd, _, RB, lsd, lsx, lsi, _ = one
    pct = S.SET_QUANTILES
    cum = np.asarray(d["cumcode"], bool)
    kw = dict(Tjumpoffs=[thisT], MCMCdraws=M, fcstNdraws=M * Nd, fcstNhorizons=H, burnin=burn, gibbsburn=5,
              nchains=C, chunk=4, cumcode=cum)
    bat = S.goVARshadowrate_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, postprocess=True, **kw)
    lite = S.goVARshadowrate_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, postprocess=False, **kw)
    assert bat["stats"]["retries"] == []

    pool = lambda a: a.reshape(a.shape[0], H, -1)                     # N x H x (draws, chains)
    yd, yz, sd = pool(fYd), pool(fYc), pool(fSd)
    yhat = RB.mean(axis=-1)
    yhat[ndxY] = yd[ndxY].mean(axis=-1)                               # mcmcVARshadowrate.m:683-684
    want = dict(fcstYhatRB=RB.mean(axis=-1), fcstYhat=yhat, fcstShadowYhat=RB.mean(axis=-1)[ndxY],
                fcstYcensorhat=yz.mean(axis=-1), fcstYrealized=yreal,
                fcstYmvlogscore=S._logmeanexp(lsd.ravel()), fcstYmvlogscoreX=S._logmeanexp(lsx.ravel()),
                fcstYmvlogscoreI=S._logmeanexp(lsi.ravel()))
    P = np.moveaxis(PAI, 3, 1).reshape(-1, *PAI.shape[1:3])          # (chains x draws) x K x N
    want.update(PAImean=P.mean(axis=0), PAIstdev=P.std(axis=0), PAImedian=np.median(P, axis=0),
                PAIquantiles=np.moveaxis(S.matlab_prctile(P, pct, axis=0), 0, 2))
    qs = lambda x: np.moveaxis(S.matlab_prctile(x, pct, axis=-1), 0, 2)
    ycum = yd.copy()
    ycum[cum] = np.cumsum(ycum[cum], axis=1)
    ycr = yreal.copy()
    ycr[cum] = np.cumsum(ycr[cum], axis=1)
    want.update(fcstYmedian=np.median(yd, axis=-1), fcstYcrps=_crps(yreal, yd), fcstYquantiles=qs(yd),
                fcstYcummedian=np.median(ycum, axis=-1), fcstYcumcrps=_crps(ycr, ycum), fcstYcumquantiles=qs(ycum),
                fcstYcensormedian=np.median(yz, axis=-1), fcstYcensorcrps=_crps(yreal, yz),
                fcstYcensorquantiles=qs(yz), fcstShadowYmedian=np.median(sd, axis=-1), fcstShadowYquantiles=qs(sd))
    jumpoff = 12 + e0
    elbT = sr.shape[2]
    assert elbT == thisT - jumpoff and elbT > 0
    shr = sr.transpose(2, 1, 0, 3).reshape(elbT, len(ndxS), -1)
    mr = miss.transpose(2, 1, 0, 3).reshape(elbT, len(ndxS), -1)
    for name, arr, mid, tails in (("shadowrate", shr, np.median(shr, axis=2), S.matlab_prctile(shr, [5, 25, 75, 95], axis=2)),
                                  ("missingrate", mr, np.median(mr, axis=2),
                                   np.nanpercentile(mr, [5, 25, 75, 95], axis=2, method="hazen"))):
        _close(name + "VintagesMid", bat[name + "VintagesMid"][jumpoff:thisT, :, 0], mid)
        _close(name + "VintagesTails", bat[name + "VintagesTails"][jumpoff:thisT, :, :, 0], np.moveaxis(tails, 0, 2))
        assert np.all(np.isnan(bat[name + "VintagesMid"][:jumpoff, :, 0]))
    assert np.all(np.isfinite(mr))                                    # every kept sweep ran the PS branch
    for k, w in want.items():
        _close(k, bat[k][..., 0], w)
    _close("fcstYcensorhaterror", bat["fcstYcensorhaterror"][..., 0], yreal - yz.mean(axis=-1))
    for k in ("fcstYhat", "fcstYhatRB", "fcstYcensorhat", "PAImean", "PAIstdev", "fcstYmvlogscore",
              "missingrateVintagesMid", "shadowrateVintagesMid"):
        _close("lite " + k, lite[k], bat[k])
    assert np.all(yd[ndxY] >= ELB) and np.all(bat["fcstYquantiles"][ndxY] >= ELB)


def test_shadowrate_batch_vintages(pkg, fred):
    """Three vintages x two chains on one set: finite scores, floors, the missingrate window."""
    S = pkg.samplers
    d = fred
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], ELB)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    nT = len(d["ydates"])
    Tj = [nT - 150, nT - 60, nT - 24]
    out = S.goVARshadowrate_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, Tjumpoffs=Tj, MCMCdraws=6, fcstNdraws=12,
                                  fcstNhorizons=12, burnin=4, gibbsburn=5, nchains=2, chunk=3)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, ELB, 12)
    assert np.all(np.isfinite(out["fcstYmvlogscore"]))
    assert np.all(out["fcstYhat"][ndxY] >= ELB) and np.all(out["fcstYcensorhat"][ndxS] >= ELB)
    assert np.all(out["countELBaccept"] >= 0)
    for v, t in enumerate(Tj):
        w = out["missingrateVintagesMid"][12 + e0:t, :, v]
        assert w.shape[0] > 0 and np.all(np.isfinite(w)), v
        assert np.all(np.isnan(out["missingrateVintagesMid"][t:, :, v]))
