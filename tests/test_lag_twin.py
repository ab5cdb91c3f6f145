"""The hybrid design is the lag structure of one (T + p) x (N + Ns) slab:
X = [1, lags 1..p of shadowYdata, lags 1..p of the actual rates floored at the ELB]
(mcmcVARhybridGibbs.m:69-84, rebuilt every sweep at :521-525), so the large path's Gram and solve
can read the column-major slab ("lag twin", ccmm_big.h ColX) instead of the K x T design.  CPU
restatement of the twin's column map (ChainSet::init_colx / try_upload_Dc in csrc/ccmm_abi.hip)
checked against the reference's own construction, before and after shadow-rate draws replace the
censored months -- every row of the sample, the ones after the shadow window included."""
import numpy as np
import pytest

from conftest import ROOT


def _twin_offsets(N, Ns, p, K, KP, ld):
    """off[a]: X(t, a) = twin[off[a] + t] (column-major, leading dimension ld)."""
    off = np.empty(KP, int)
    for a in range(KP):
        if a == 0:
            off[a] = (N + Ns) * ld                     # the column of ones
        elif a >= K:
            off[a] = (N + Ns + 1) * ld                 # the zero column (padded coefficients)
        elif a - 1 < N * p:
            b = a - 1
            off[a] = (b % N) * ld + p - (b // N + 1)   # lag l of variable k
        else:
            b = a - 1 - N * p
            off[a] = (N + b % Ns) * ld + p - (b // Ns + 1)  # lag l of actual rate s
    return off


def _twin(slab, ld):
    """Column-major twin of the (Nobs x (N + Ns)) slab: rows 0..Nobs-1, then ones and zeros."""
    Nobs, nc = slab.shape
    D = np.zeros((nc + 2) * ld)
    for k in range(nc):
        D[k * ld:k * ld + Nobs] = slab[:, k]
    D[nc * ld:(nc + 1) * ld] = 1.0
    return D


def _reference_x(data, ndxS, p, ELB):
    """mcmcVARhybridGibbs.m:69-84 / :521-525 as written (0-based)."""
    Nobs, N = data.shape
    lags = np.zeros((Nobs, N * p))
    for l in range(1, p + 1):
        lags[p:, N * (l - 1):N * l] = data[p - l:Nobs - l, :]
    Ns = len(ndxS)
    ffr = np.zeros((Nobs, p * Ns))
    for l in range(1, p + 1):
        ffr[p:, (l - 1) * Ns:l * Ns] = data[p - l:Nobs - l][:, ndxS]
    xffr = ffr[p:, :].copy()
    xffr[xffr < ELB] = ELB
    return np.hstack([np.ones((Nobs - p, 1)), lags[p:, :], xffr])


@pytest.mark.parametrize("draws", [False, True])
def test_hybrid_design_is_the_lags_of_one_slab(pkg, draws):
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, _, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    hm = pkg.model.build_hybrid(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, mpm, 0.25, e0, True)
    m = hm.var
    N, Ns, T, K = m.N, len(hm.ndxS), m.T, m.K
    data = np.array(m.data, float)
    X = m.X
    if draws:
        # shadow-rate draws in the window (elbT0 + 1 .. T): shadowYdata(p+elbT0+1:end, ndxS) (:498);
        # the actual-rate block keeps the data (Xffrlags is built once, :81-84)
        rng = np.random.default_rng(5)
        data[p + hm.elbT0:, hm.ndxS] = rng.normal(-1.0, 1.0, (T - hm.elbT0, Ns))
        X = _reference_x(data, hm.ndxS, p, 0.25)
        X[:, 1 + N * p:] = m.X[:, 1 + N * p:]
    else:
        np.testing.assert_array_equal(X, _reference_x(data, hm.ndxS, p, 0.25))
    KP = -(-K // 64) * 64
    TP = -(-T // 32) * 32
    ld = -(-(TP + p) // 8) * 8
    actual = np.where(np.array(m.data)[:, hm.ndxS] < 0.25, 0.25, np.array(m.data)[:, hm.ndxS])
    slab = np.hstack([data, actual])
    D = _twin(slab, ld)
    off = _twin_offsets(N, Ns, p, K, KP, ld)
    t = np.arange(T)
    for a in range(K):
        np.testing.assert_array_equal(D[off[a] + t], X[:, a], err_msg=f"column {a}")
    assert np.all(D[off[K:KP, None] + np.arange(TP)[None, :]] == 0.0)     # padded coefficients read zeros
    assert off.max() + TP <= D.size                                       # every read inside the slab


def test_linear_design_is_the_lags_of_its_data(pkg):
    """mcmcVAR.m:62-72: the linear model's X is the N-column case of the same map (S120's large path)."""
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    m = pkg.model.build_var(len(d["ydates"]), p, 12, d["data"], d["ydates"], mpm, True)
    N, T, K = m.N, m.T, m.K
    KP = -(-K // 64) * 64
    ld = -(-(-(-T // 32) * 32 + p) // 8) * 8
    D = np.zeros((N + 2) * ld)
    for k in range(N):
        D[k * ld:k * ld + T + p] = np.asarray(m.data, float)[:T + p, k]
    D[N * ld:(N + 1) * ld] = 1.0
    off = _twin_offsets(N, 0, p, K, KP, ld)
    t = np.arange(T)
    for a in range(K):
        np.testing.assert_array_equal(D[off[a] + t], m.X[:, a], err_msg=f"column {a}")
