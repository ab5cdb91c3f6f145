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
