"""GPU parity of the per-vintage post-processing (goVARshadowrateBlockHybrid.m:349-480;
ccmm_post.hip: gather, rocPRIM segmented sort, summary kernel) against the oracle
(oracle/ccmm_oracle_post.py: MATLAB prctile / median / std(.,1) / crpsDraws).

Order statistics (median, quantiles) are compared bit for bit: the kernel reproduces
numpy's index and interpolation arithmetic.  Sums (mean, std, CRPS) are reduced in a
different order than numpy's pairwise summation: 1e-13 relative.

CRPS parity is UNPINNED: crpsDraws lives in the absent em-matlabbox submodule, so the oracle's
estimator (the CRPS of the draws' empirical distribution, mean|x - y| - sum_i (2i - n - 1) x_(i) / n^2,
Gneiting-Raftery eq. 21) is a declared convention that the device matches; an estimator with
1 / (n (n - 1)) would give different values and no reference output decides between them."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def post():
    from oracle import ccmm_oracle_post
    return ccmm_oracle_post


def _cmp_sums(got, want, tol=1e-13):
    assert np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)) < tol


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 10000, 25001])
def test_draw_summaries(ctx, post, n):
    rng = np.random.default_rng(n)
    S = 13
    X = rng.standard_normal((n, S)) * np.linspace(0.1, 5, S) + np.linspace(-3, 3, S)
    X[: n // 3, 0] = 0.25                      # ties (censored paths sit at the ELB)
    X[:, 1] = np.round(X[:, 1], 1)             # many ties
    X[:, 2] = -0.0 if n % 2 else 0.0
    y = rng.standard_normal(S)
    y[3] = np.nan
    pct = post.SET_QUANTILES
    got = ctx.draw_summaries(X, realized=y, pct=pct)
    assert np.array_equal(got["median"], post.median(X, 0))
    assert np.array_equal(got["quantiles"], np.moveaxis(post.prctile(X, pct, 0), 0, 1))
    _cmp_sums(got["mean"], X.mean(axis=0))
    _cmp_sums(got["stdev"], post.std1(X, 0))
    want = post.crps_draws(y, X.T)
    assert np.isnan(got["crps"][3]) and np.isnan(want[3])
    m = ~np.isnan(want)
    _cmp_sums(got["crps"][m], want[m], 1e-12)


def test_chain_set_summaries_bh(pkg, ctx, oracle, post):
    """Device summaries over a block-hybrid chain set's kept forecast paths (censored,
    cumulated, shadow-rate rows) and PAI draws equal the oracle's on the same draws."""
    from oracle import ccmm_oracle_bh as bh
    from helpers import toy_bh_setup
    bs = toy_bh_setup(bh)
    lin = bs.lin
    N, H, Nd, M, B = lin.N, 6, 3, 4, 3
    ch = pkg.Chains(ctx, N=N, p=lin.p, T=lin.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=3, elb=bs.ELB,
                    store_capacity=M, seed=9)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    yields = np.zeros(N, bool)
    yields[[2, 3, 4]] = True
    ch.set_fcst(H, Nd, yields, keep_paths=True)
    yr = np.random.default_rng(1).standard_normal((N, H))
    ch.set_fcst_slot(0, yr[:, 0])
    st = oracle.init_state(lin)
    ch.set_state(*[np.repeat(st[k][..., None], B, -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    ch.sweep(2, store=False)
    ch.sweep(M, store=True)
    pct = post.SET_QUANTILES
    cum = np.array([True, False, False, True, False])
    yd = ch.summaries(1, 0, realized=yr, pct=pct)
    ycr = yr.copy()
    ycr[cum] = np.cumsum(ycr[cum], axis=1)
    yc = ch.summaries(1, 0, cumcode=cum, realized=ycr, pct=pct)
    sh = ch.summaries(0, 0, rows=yields, pct=pct)
    pa = ch.summaries(2, 0, pct=pct)
    fc = ch.get_fcst(paths=True)
    dr = ch.get_draws()
    D = M * Nd * B
    ydraws = fc["paths_censored"].reshape(N, H, -1, order="F")     # N x H x (job, m, c)
    assert ydraws.shape[2] == D
    ycum = ydraws.copy()
    ycum[cum] = np.cumsum(ycum[cum], axis=1)
    sdraws = fc["paths"].reshape(N, H, -1, order="F")[yields]
    for got, draws, real in ((yd, ydraws, yr), (yc, ycum, ycr), (sh, sdraws, None)):
        S = draws.shape[0] * H
        flat = draws.reshape(S, -1, order="F").T        # n x S, series = row + nr h
        assert np.array_equal(got["median"], post.median(flat, 0))
        assert np.array_equal(got["quantiles"], np.moveaxis(post.prctile(flat, pct, 0), 0, 1))
        _cmp_sums(got["mean"], flat.mean(axis=0))
        if real is not None:
            _cmp_sums(got["crps"], post.crps_draws(real.ravel(order="F"), flat.T), 1e-12)
    P = dr["PAI_all"].transpose(0, 3, 1, 2).reshape(M * B, lin.K * N, order="F")
    assert np.array_equal(pa["median"], post.median(P, 0))
    assert np.array_equal(pa["quantiles"], np.moveaxis(post.prctile(P, pct, 0), 0, 1))
    _cmp_sums(pa["stdev"], post.std1(P, 0), 1e-10)
    ch.close()


def test_batch_postprocess_small(pkg, fred, tmp_path):
    """goVARshadowrateBlockHybrid_batch(postprocess=True) over three vintages: every
    per-vintage summary present and finite, the CRPS non-negative, and the QRT .mat file
    written (save_qrt_mat)."""
    S = pkg.samplers
    ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    Tj = [len(fred["ydates"]) - 40, len(fred["ydates"]) - 20, len(fred["ydates"])]
    res = S.goVARshadowrateBlockHybrid_batch(fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                                             Tjumpoffs=Tj, MCMCdraws=8, fcstNdraws=16, burnin=6,
                                             gibbsburn=5, nchains=2, chunk=4, postprocess=True,
                                             cumcode=fred["cumcode"], maxlambda=True, Nproposals=50)
    V, N, H = 3, 20, 48
    assert res["fcstYquantiles"].shape == (N, H, 10, V)
    assert res["PAIquantiles"].shape == (241, N, 10, V)
    for k in ("fcstYmedian", "fcstYquantiles", "fcstYcumhat", "fcstYcummedian", "PAImedian",
              "fcstShadowYmedian", "drawsMaxVARroot"):
        assert np.all(np.isfinite(res[k])), k
    crps = res["fcstYcrps"]
    fin = np.isfinite(crps)
    assert fin[:, :8, :2].all() and np.all(crps[fin] >= -1e-12)
    q = res["fcstYquantiles"]
    assert np.all(np.diff(q, axis=2) >= 0)                     # quantiles ordered
    assert res["fcstYmvlogscoreDraws"].shape == (16 * 2, V)
    names = S.save_qrt_mat(tmp_path / "qrt.mat", res, data=fred["data"], ydates=fred["ydates"], p=12,
                           ncode=fred["ncode"], tcode=fred["tcode"], cumcode=fred["cumcode"],
                           ndxSHADOWRATE=ndxS, ndxOTHERYIELDS=ndxO, ELBbound=0.25,
                           actualrateBlock=~np.isin(np.arange(N), np.union1d(ndxS, ndxO)),
                           datalabel="fredblockMD20-2022-09", modellabel="ELBblockhybrid",
                           MCMCdraws=8, fcstNhorizons=H)
    assert "fcstYcrps" in names and "PAIquantiles" in names
