"""CPU checks of the oracle's momentg (Diagnostics.m:134-300) restatement: the vectorised
form equals a loop-by-loop transcription of the MATLAB on random data, and its NSE behave
as Geweke's estimator should (iid: all tapers ~ pstd / sqrt(n); AR(1): tapers grow)."""
import numpy as np

from oracle.ccmm_oracle_stats import momentg


def _momentg_loops(d):
    """Diagnostics.m:182-297 statement by statement (one variable; ad = 1)."""
    NG = 100
    ndraw = len(d)
    ns = ndraw // NG
    nuse = ns * NG
    cn, cd = np.zeros(NG), np.zeros(NG)
    td = tn = tdd = tnn = tdn = tvar = 0.0
    cnt = 0
    for ig in range(NG):
        gd = gn = gdd = gdn = gnn = gvar = 0.0
        for _ in range(ns):
            g = d[cnt]
            cnt += 1
            ad = 1.0
            an = ad * g
            gd += ad
            gn += an
            gdn += ad * an
            gdd += ad * ad
            gnn += an * an
            gvar += an * g
        td += gd
        tn += gn
        tdn += gdn
        tdd += gdd
        tnn += gnn
        tvar += gvar
        cn[ig] = gn / ns
        cd[ig] = gd / ns
    eg = tn / td
    varg = tvar / td - eg ** 2
    res = {"pmean": eg, "pstd": np.sqrt(varg)}
    varnum = (tnn - 2 * eg * tdn + tdd * eg ** 2) / td ** 2
    res["nse"] = np.sqrt(varnum)
    barn, bard = tn / nuse, td / nuse
    cn -= barn
    cd -= bard
    rnn, rdd, rnd = np.zeros(NG), np.zeros(NG), np.zeros(NG)
    for lag in range(NG):
        ann = add = and_ = 0.0
        for ig in range(lag, NG):
            ann += cn[ig] * cn[ig - lag]
            add += cd[ig] * cd[ig - lag]
            and_ += cn[ig] * cd[ig - lag]
        rnn[lag], rdd[lag], rnd[lag] = ann / NG, add / NG, and_ / NG
    for k, m in enumerate((4, 8, 15), start=1):
        snn, sdd, snd = rnn[0], rdd[0], rnd[0]
        for lag in range(1, m):
            att = 1 - lag / m
            snn += 2 * att * rnn[lag]
            sdd += 2 * att * rdd[lag]
            snd += att * (rnd[lag] + rnd[lag])
        varnum = ns * nuse * (snn - 2 * eg * snd + sdd * eg ** 2) / td ** 2
        res[f"nse{k}"] = np.sqrt(varnum)
    return res


def test_momentg_matches_loops():
    rng = np.random.default_rng(1)
    D = np.cumsum(rng.standard_normal((537, 3)), axis=0) * 0.1 + rng.standard_normal((537, 3))
    v = momentg(D)
    for j in range(3):
        ref = _momentg_loops(D[:, j])
        for k in ("pmean", "pstd", "nse", "nse1", "nse2", "nse3"):
            assert abs(v[k][j] - ref[k]) <= 1e-12 * max(1.0, abs(ref[k])), (k, v[k][j], ref[k])


def test_momentg_iid_and_ar1():
    rng = np.random.default_rng(2)
    n = 20000
    iid = rng.standard_normal(n)
    v = momentg(iid)
    for k in ("nse", "nse1", "nse2", "nse3"):
        assert abs(v[k][0] * np.sqrt(n) - 1.0) < 0.5  # 100 group means: the tapered estimates are noisy
    x = np.empty(n)
    x[0] = 0.0
    e = rng.standard_normal(n)
    for t in range(1, n):
        x[t] = 0.9 * x[t - 1] + e[t]
    w = momentg(x)
    # long-run sd of an AR(1) mean is sd / (1 - rho) per sqrt(n): the tapered estimates grow
    # toward it, the iid one does not
    assert w["nse3"][0] > 2.5 * w["nse"][0]


def test_psrf_known_answer():
    """psrf (DiagnosticsShadowrate.m:34-128) by hand: one chain 1..9 -> thirds [1 2 3], [7 8 9]:
    W = 1, Bpn = 18, S = 2/3 + 18, R = sqrt(3/2 S - 1/3) = sqrt(83/3)."""
    from oracle.ccmm_oracle_stats import psrf, diagnostics_shadowrate
    assert abs(psrf(np.arange(1.0, 10.0))[0] - np.sqrt(83.0 / 3.0)) < 1e-14
    # floor(10/3) = 3: [1 2 3] and the last three [8 9 10], Bpn = 2 * 3.5^2
    assert abs(psrf(np.arange(1.0, 11.0))[0] - np.sqrt(1.5 * (2.0 / 3.0 + 24.5) - 1.0 / 3.0)) < 1e-14
    # M sequences: R^2 = (M+1)/M S/W - (n-1)/(M n), S = (n-1)/n W + B/n
    rng = np.random.default_rng(3)
    X = rng.standard_normal((50, 2, 4)) + np.array([0.0, 0.3, -0.2, 0.5])[None, None, :]
    n, M = 50, 4
    for d in range(2):
        x = X[:, d, :]
        W = x.var(axis=0, ddof=1).mean()
        B = n * x.mean(axis=0).var(ddof=1)
        S = (n - 1) / n * W + B / n
        assert abs(psrf(X)[d] - np.sqrt((M + 1) / M * S / W - (n - 1) / (M * n))) < 1e-13
    # iid draws: R -> 1; no cells: NaN (mean of an empty row)
    assert abs(diagnostics_shadowrate(rng.standard_normal((30000, 3))) - 1.0) < 0.01
    assert np.isnan(diagnostics_shadowrate(np.zeros((300, 0))))
