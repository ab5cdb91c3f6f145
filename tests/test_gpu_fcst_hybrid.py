"""GPU parity of the hybrid model's predictive density (mcmcVARhybridGibbs.m:566-635 and the
censoring of :703-711) computed inside the chain set (ccmm_chains_set_fcst, k_fcst hybrid mode)
against oracle/ccmm_oracle_fcst.fcst_draw_hybrid (the dense companion on Kshadow + Ns p states
with fcstA(ndxfcstY,:) = PAI', actual-rate states max(shadow, ELB), as written) on the GPU's
own post-sweep state, two real-data vintages in one chain set: an ELB-era jump-off with the
three shadow rates realized at the ELB (censored trivariate score) and a 2017 jump-off with
none.  Paths 1e-9 in |Δ| / max(|x|, 1); scores 1e-9 (1e-8 with three series at the ELB)."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

H, ND = 12, 5


@pytest.fixture(scope="module")
def F():
    from oracle import ccmm_oracle_fcst
    return ccmm_oracle_fcst


def test_hybrid_chain_fcst_two_vintages(pkg, ctx, fred, F):
    p = 12
    d = fred
    nT = len(d["ydates"])
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    vint = []
    for thisT in (585 + p + 1 + 40, nT - 60):
        hm = pkg.model.build_hybrid(thisT, p, 12, d["data"], d["ydates"], ndxS, mpm, 0.25, e0, True)
        yr = pkg.samplers.realized_values(d["data"], thisT, H, ndxS, 0.25)
        vint.append((thisT, hm, yr))
    C = 2
    B = C * len(vint)
    Tmax = max(v[1].var.T for v in vint)
    elbTmax = max(v[1].elbT for v in vint)
    m0 = vint[0][1]
    N, K = m0.var.N, m0.var.K
    ch = pkg.Chains(ctx, N=N, p=p, T=Tmax, B=B, ndata=len(vint), crn=True, model=pkg.MODEL_HYBRID,
                    Ns=len(ndxS), elbTmax=elbTmax, elb_gibbsburn=20, elb=0.25, store_capacity=2)
    for s, (thisT, hm, yr) in enumerate(vint):
        m = hm.var
        ch.set_data(s, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(m0.ndxS, None)
    yields = np.zeros(N, bool)
    yields[ndxY] = True
    ch.set_fcst(H, ND, yields, keep_paths=True)
    slots = np.repeat(np.arange(len(vint)), C)
    ch.set_slots(slots)
    init = {k: np.zeros(sh) for k, sh in (("PAI", (K, N, B)), ("A", (N, N, B)), ("sqrtht", (Tmax, N, B)),
                                           ("h", (Tmax, N, B)), ("sqrtPHI", (N, N, B)))}
    for s, (thisT, hm, yr) in enumerate(vint):
        ch.set_elb_slot(s, hm.elbT0, hm.sNaN)
        ch.set_fcst_slot(s, yr[:, 0])
        st = pkg.model.initial_state(hm.var, C)
        T = hm.var.T
        for k in init:
            v = st[k]
            if k in ("sqrtht", "h"):
                pad = np.ones((Tmax - T,) + v.shape[1:]) if k == "sqrtht" else np.zeros((Tmax - T,) + v.shape[1:])
                v = np.concatenate([v, pad], axis=0)
            init[k][..., s * C:(s + 1) * C] = v
    ch.set_state(init["PAI"], init["A"], init["sqrtht"], init["h"], init["sqrtPHI"])
    rng = np.random.default_rng(13)
    crn = ch.draw_crn(rng, 2)
    ch.sweep(1, crn=crn[:, :1], store=False)
    ch.sweep(1, crn=crn[:, 1:], store=True)
    st = ch.get_state()
    X, Y = ch.get_xy()
    fc = ch.get_fcst(paths=True)
    assert fc["M"] == 1 and not fc["warn_mvncdf"]
    off, n, _ = ch.crn_layout()["FCST"]
    ch.close()
    nat_seen = set()
    for c in range(B):
        thisT, hm, yr = vint[slots[c]]
        T = hm.var.T
        Xj = F.hybrid_jumpoff(Y[:T, :, c], d["data"][:thisT], p, ndxS, 0.25)
        seg = crn[off:off + n, 1, c]
        svz = seg[:N * H * ND].reshape(N, H * ND, order="F")
        z = seg[N * H * ND:].reshape(N, H, ND, order="F")
        fY, sc = F.fcst_draw_hybrid(st["PAI"][..., c], st["invA"][..., c], st["h"][T - 1, :, c],
                                    st["sqrtPHI"][..., c], Xj, yr[:, 0], yields, ndxS, 0.25, svz, z)
        e = rel_err(fc["paths"][..., 0, c], fY, 1.0)
        assert e < 1e-9, (c, e)
        fYc = fY.copy()
        fYc[yields] = np.maximum(fYc[yields], 0.25)                   # :707-711
        assert rel_err(fc["paths_censored"][..., 0, c], fYc, 1.0) < 1e-9
        nat = int(np.sum(yr[yields, 0] <= 0.25))
        nat_seen.add(nat)
        gsc = fc["scores"][:, 0, :, c]
        tol = 1e-8 if nat == 3 else 1e-9
        for k_dev, k_or in ((1, 0), (2, 1), (3, 2)):
            e = rel_err(gsc[:, k_dev], sc[k_or], 1.0)
            print("hybrid fcst chain", c, "score", k_dev, e)
            assert e < tol, (c, k_dev, e)
    assert nat_seen == {0, 3}, nat_seen


def test_mcmcVARhybridGibbs_predictive_density(pkg, fred):
    """The reference-interface mirror with fcstNdraws: outputs 7-13 of mcmcVARhybridGibbs.m
    (fcstYdraws censored, fcstYhat, fcstShadowrateDraws, fcstShadowrateHat, the three
    one-step score draws), shapes and the ELB floor."""
    p = 12
    d = fred
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    thisT = 585 + p + 1 + 40
    yr = pkg.samplers.realized_values(d["data"], thisT, 8, ndxS, 0.25)
    out = pkg.samplers.mcmcVARhybridGibbs(thisT, 4, p, 12, d["data"], d["ydates"], None, mpm, True, ndxS, ndxO,
                                          True, False, 0.25, e0, yrealized=yr, fcstNdraws=12, fcstNhorizons=8,
                                          burnin=3, gibbsburn=5, Nproposals=50)
    fYd, fYhat, fSd, fShat, ls, lsX, lsI = out[6:13]
    N = d["data"].shape[1]
    assert fYd.shape == (N, 8, 12) and fSd.shape == (len(ndxY), 8, 12)
    assert np.all(fYd[ndxY] >= 0.25) and np.all(np.isfinite(fYd))
    np.testing.assert_allclose(fYhat, fYd.mean(axis=2))
    np.testing.assert_allclose(fShat, fSd.mean(axis=2))
    assert ls.shape == (12,) and np.all(np.isfinite(ls)) and np.all(np.isfinite(lsX))


def test_goVARhybrid_batch_small(pkg, fred, tmp_path):
    """goVARhybrid_batch (goVARhybrid.m:126-517: mcmcVARhybridGibbs per vintage) over three
    vintages x 2 chains with the device post-processing: per-vintage log scores and summaries
    finite, PAI summaries over K = N p + 1 + Ns p, the QRT file written as ELBhybrid."""
    S = pkg.samplers
    d = fred
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    nT = len(d["ydates"])
    Tj = [nT - 120, nT - 40, nT - 10]
    res = S.goVARhybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, Tjumpoffs=Tj, MCMCdraws=6, fcstNdraws=12,
                              burnin=4, gibbsburn=5, nchains=2, chunk=3, postprocess=True, cumcode=d["cumcode"],
                              Nproposals=50)
    N, H, V = 20, 48, 3
    K = N * 12 + 1 + len(ndxS) * 12
    assert res["PAImean"].shape == (K, N, V) and res["PAIquantiles"].shape == (K, N, 10, V)
    for k in ("fcstYmvlogscore", "fcstYmvlogscoreX", "fcstYmvlogscoreI", "fcstYmedian", "fcstYhat", "PAImedian"):
        assert np.all(np.isfinite(res[k])), k
    assert np.all(res["fcstYquantiles"][ndxS] >= 0.25)
    names = S.save_qrt_mat(tmp_path / "qrt.mat", res, data=d["data"], ydates=d["ydates"], p=12, ncode=d["ncode"],
                           tcode=d["tcode"], cumcode=d["cumcode"], ndxSHADOWRATE=ndxS, ndxOTHERYIELDS=ndxO,
                           ELBbound=0.25, actualrateBlock=np.zeros(N, bool), datalabel="fredblockMD20-2022-09",
                           modellabel="ELBhybrid", MCMCdraws=6, fcstNhorizons=H)
    assert "fcstYmvlogscore" in names and "PAIquantiles" in names
