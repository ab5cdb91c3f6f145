"""CPU checks of the post-processing oracle (oracle/ccmm_oracle_post.py, the restatement of
goVARshadowrateBlockHybrid.m:349-480) and of the QRT .mat writer (:641-669)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def post():
    from oracle import ccmm_oracle_post
    return ccmm_oracle_post


def test_crps_draws_matches_pair_form(post):
    """Sorted-draw form == mean|x - y| - sum_ij |x_i - x_j| / (2 n^2)."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((4, 301))
    x[0, :10] = 0.5                                   # ties
    y = np.array([0.1, -2.0, 5.0, 0.5])
    got = post.crps_draws(y, x)
    for s in range(4):
        pair = np.abs(x[s][:, None] - x[s][None, :]).sum() / (2 * x.shape[1] ** 2)
        want = np.mean(np.abs(x[s] - y[s])) - pair
        assert abs(got[s] - want) < 1e-12
    assert np.isnan(post.crps_draws(np.nan, x[0]))


def test_prctile_matlab_definition(post):
    """prctile: the i-th sorted value at percentile 100 (i - 0.5)/n, linear between,
    extremes outside."""
    rng = np.random.default_rng(4)
    x = rng.standard_normal(57)
    xs = np.sort(x)
    n = x.size
    for pc in list(post.SET_QUANTILES) + [0.0, 0.3, 50.0, 99.9, 100.0]:
        r = n * pc / 100 + 0.5                            # 1-based position
        if r <= 1:
            want = xs[0]
        elif r >= n:
            want = xs[-1]
        else:
            k = int(np.floor(r))
            want = xs[k - 1] + (r - k) * (xs[k] - xs[k - 1])
        assert abs(post.prctile(x, pc) - want) < 1e-14
    assert post.median(np.array([1.0, 4.0, 2.0, 3.0])) == 2.5


def test_vma_and_sum_ffr(post):
    rng = np.random.default_rng(5)
    N, p, H = 3, 2, 6
    PAI = 0.2 * rng.standard_normal((1 + N * p, N))
    v = post.vma(PAI, N, p, H)
    Phi = [PAI[1 + l * N:1 + (l + 1) * N, :].T for l in range(p)]
    psi = [np.eye(N)]
    for h in range(1, H + 1):
        psi.append(sum(Phi[l] @ psi[h - 1 - l] for l in range(p) if h - 1 - l >= 0))
    for h in range(H):
        assert np.allclose(v[:, :, h], psi[h + 1], atol=1e-14)
    assert np.allclose(post.sum_ffr(PAI, N, p, 1), PAI[[2, 2 + N], :].sum(axis=0))


def test_save_qrt_mat_roundtrip(pkg, tmp_path):
    from scipy.io import loadmat
    S = pkg.samplers
    N, H, V, K, Ns, T = 4, 3, 2, 9, 2, 30
    rng = np.random.default_rng(6)
    res = dict(Tjumpoffs=np.array([25, 26]), fcstYhat=rng.standard_normal((N, H, V)),
               fcstYmvlogscore=rng.standard_normal(V), PAImean=rng.standard_normal((K, N, V)),
               shadowrateVintagesMid=rng.standard_normal((T, Ns, V)))
    data = rng.standard_normal((T, N))
    names = S.save_qrt_mat(tmp_path / "q.mat", res, data=data, ydates=np.arange(T), p=2,
                           ncode=["A", "B", "FEDFUNDS", "GS10"], tcode=[5, 5, 1, 1],
                           cumcode=[True, True, False, False], ndxSHADOWRATE=[2],
                           ndxOTHERYIELDS=[3], ELBbound=0.25,
                           actualrateBlock=[True, True, False, False], datalabel="toy",
                           modellabel="ELBblockhybrid", MCMCdraws=10, fcstNhorizons=H)
    m = loadmat(tmp_path / "q.mat")
    for k in ("fcstYhat", "PAImean", "shadowrateVintagesMid", "setQuantiles", "ndxSHADOWRATE"):
        assert k in names and k in m
    assert np.allclose(m["fcstYhat"], res["fcstYhat"])
    assert m["ndxSHADOWRATE"].ravel().tolist() == [3]      # 1-based
    assert m["fcstYmvlogscore"].shape == (1, V)


def test_matlab_prctile_removes_nan(pkg, post):
    """samplers.matlab_prctile (shadowrate* and missingrate* tails, goVARshadowrate.m:345-348) drops
    NaN draws as MATLAB prctile does: equal to the written-out definition on the remaining values."""
    S = pkg.samplers
    rng = np.random.default_rng(8)
    x = rng.standard_normal((5, 3, 41))
    x[0, 0, :7] = np.nan
    x[1, 2, ::3] = np.nan
    x[2, 1, :] = np.nan                                # all NaN: NaN
    got = np.moveaxis(S.matlab_prctile(x, [5, 25, 75, 95], axis=2), 0, 2)
    for i in range(5):
        for j in range(3):
            want = post.prctile_nan(x[i, j], [5, 25, 75, 95])
            assert np.array_equal(np.isnan(got[i, j]), np.isnan(want))
            m = ~np.isnan(want)
            assert np.allclose(got[i, j][m], want[m], rtol=0, atol=1e-14)
    y = rng.standard_normal((4, 30))                   # no NaN: the plain hazen path
    assert np.allclose(S.matlab_prctile(y, [2.5, 50], axis=1).T,
                       [post.prctile_nan(r, [2.5, 50]) for r in y], rtol=0, atol=1e-14)


def test_save_qrt_mat_varlist_has_psrf(pkg, tmp_path):
    """The saved file holds every name of goVARshadowrateBlockHybrid.m:645-659's varlist that the batch
    result carries, shadowratePSRF (Nshadowrates x Njumpoffs, :213) among the 'shadowrate*' names."""
    from scipy.io import loadmat
    S = pkg.samplers
    N, H, V, Ns, T = 4, 3, 2, 2, 30
    rng = np.random.default_rng(9)
    res = dict(Tjumpoffs=np.array([25, 26]), fcstYhat=rng.standard_normal((N, H, V)),
               shadowratePSRF=1.0 + rng.random((Ns, V)), shadowrateVintagesMid=rng.standard_normal((T, Ns, V)))
    names = S.save_qrt_mat(tmp_path / "q.mat", res, data=rng.standard_normal((T, N)), ydates=np.arange(T), p=2,
                           ncode=["A", "FEDFUNDS", "GS1", "GS10"], tcode=[5, 1, 1, 1],
                           cumcode=[True, False, False, False], ndxSHADOWRATE=[1, 2], ndxOTHERYIELDS=[3],
                           ELBbound=0.25, actualrateBlock=[True, False, False, False], datalabel="toy",
                           modellabel="ELBblockhybrid", MCMCdraws=10, fcstNhorizons=H)
    m = loadmat(tmp_path / "q.mat")
    assert "shadowratePSRF" in names and m["shadowratePSRF"].shape == (Ns, V)
    assert np.allclose(m["shadowratePSRF"], res["shadowratePSRF"])
    fixed = {"data", "ydates", "p", "Tjumpoffs", "N", "ncode", "tcode", "cumcode", "fcstNhorizons",
             "ndxSHADOWRATE", "ndxYIELDS", "ndxOTHERYIELDS", "ELBbound", "ELBdummy", "actualrateBlock",
             "datalabel", "modellabel", "doQuarterly", "setQuantiles", "MCMCdraws"}
    assert fixed <= set(names)
