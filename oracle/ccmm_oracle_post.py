"""Oracle (CPU restatement) of the per-vintage post-processing of the quasi-real-time
OOS driver goVARshadowrateBlockHybrid.m:318-514 — TEST INFRASTRUCTURE ONLY (the
device path is ccmm_post.hip via ccmm_draw_summaries / ccmm_chains_summaries).

MATLAB semantics restated:
  prctile(x, p, dim)  (Statistics Toolbox): the sorted sample's i-th value sits at
      percentile 100 (i - 0.5) / n; linear interpolation in between, the extremes outside
      (= numpy method "hazen"); median = prctile 50 (the mean of the middle pair for even n)
  std(x, 1, dim)      normalised by n
  crpsDraws(y, draws) (em-matlabbox, source absent — PARITY UNPINNED): the CRPS of the
      empirical distribution of the draws, mean|x - y| - 1/(2 n^2) sum_ij |x_i - x_j|
      (Gneiting & Raftery 2007 eq. 21; Krueger et al. 2021 "CRPS_ECDF"), evaluated from the
      sorted draws as mean|x - y| - 1/n^2 sum_i (2 i - n - 1) x_(i)
  max(abs(eig(comp)))  companion matrix of PAI(2:Kbvar,:)' (:384-392)
"""
from __future__ import annotations

import numpy as np

SET_QUANTILES = None  # filled below: goVARshadowrateBlockHybrid.m:141


def _normcdf(x):
    from math import erfc, sqrt
    return 0.5 * erfc(-x / sqrt(2.0))


SET_QUANTILES = np.array([.5, 2.5, 5, _normcdf(-1) * 100, 25, 75, (1 - _normcdf(-1)) * 100, 95,
                          97.5, 99.5])


def prctile(x, pct, axis=0):
    """MATLAB prctile along ``axis``; returns the percentile axis first when pct is a list."""
    return np.percentile(np.asarray(x, float), pct, axis=axis, method="hazen")


def prctile_nan(x, pct):
    """MATLAB prctile of one vector with NaN values removed first (prctile ignores NaN; all NaN:
    NaN), written out: the i-th of the n sorted values at percentile 100 (i - 0.5) / n."""
    xs = np.sort(np.asarray(x, float)[~np.isnan(np.asarray(x, float))])
    n = xs.size
    out = []
    for pc in np.atleast_1d(pct):
        if n == 0:
            out.append(np.nan)
            continue
        r = n * pc / 100.0 + 0.5                     # 1-based position
        if r <= 1:
            out.append(xs[0])
        elif r >= n:
            out.append(xs[-1])
        else:
            k = int(np.floor(r))
            out.append(xs[k - 1] + (r - k) * (xs[k] - xs[k - 1]))
    return np.array(out)


def median(x, axis=0):
    return np.median(np.asarray(x, float), axis=axis)


def std1(x, axis=0):
    """std(x, 1, axis): normalised by n."""
    return np.std(np.asarray(x, float), axis=axis)


def crps_draws(y, draws, axis=-1):
    """crpsDraws(y, draws): CRPS of the empirical distribution of ``draws`` along ``axis``
    at the realisation y (NaN y gives NaN).  PARITY UNPINNED: em-matlabbox's crpsDraws source is
    absent; this is the declared estimator (1 / n^2 normalisation, Gneiting-Raftery eq. 21)."""
    x = np.sort(np.moveaxis(np.asarray(draws, float), axis, -1), axis=-1)
    n = x.shape[-1]
    y = np.asarray(y, float)[..., None]
    w = (2.0 * np.arange(1, n + 1) - n - 1.0)
    return np.mean(np.abs(x - y), axis=-1) - (x @ w) / (n * n)


def companion(PAI, N, p):
    """comp of :384-392: first N rows PAI(2:Kbvar,:)', identity below."""
    comp = np.zeros((N * p, N * p))
    comp[N:, :N * (p - 1)] = np.eye(N * (p - 1))
    comp[:N, :] = PAI[1:1 + N * p, :].T
    return comp


def max_var_root(PAI_all, N, p):
    """theseMaxlambdas(m) = max(abs(eig(comp))) over the draws (:387-392)."""
    return np.array([np.max(np.abs(np.linalg.eigvals(companion(P, N, p)))) for P in PAI_all])


def vma(PAI, N, p, H):
    """drawsVMA(:,:,h) = (comp^h)(1:N, 1:N), h = 1..H (:397-408)."""
    comp = companion(PAI, N, p)
    out = np.zeros((N, N, H))
    cp = np.eye(N * p, N)
    for h in range(H):
        cp = comp @ cp
        out[:, :, h] = cp[:N, :N]
    return out


def sum_ffr(PAI, N, p, ffr):
    """sumFFR(:, m) = sum over lags of the FEDFUNDS coefficients (:416-425), ffr 0-based."""
    rows = [1 + l * N + ffr for l in range(p)]
    return PAI[rows, :].sum(axis=0)


def vintage_summaries(ydraws, yhat, yrealized, shadowdraws, shadowhat, cumcode, PAI_all, N, p,
                      pct=SET_QUANTILES):
    """The per-vintage block :349-480 for one vintage.
    ydraws N x H x D, yhat N x H, yrealized N x H, shadowdraws Ny x H x D, shadowhat Ny x H,
    cumcode bool N, PAI_all M x K x N."""
    cc = np.asarray(cumcode, bool)
    ycumrealized = np.array(yrealized, float)
    ycumdraws = np.array(ydraws, float)
    ycumhat = np.array(yhat, float)
    ycumrealized[cc] = np.cumsum(ycumrealized[cc], axis=1)                         # :353
    ycumdraws[cc] = np.cumsum(ycumdraws[cc], axis=1)                               # :354
    ycumhat[cc] = np.cumsum(ycumhat[cc], axis=1)                                   # :355
    out = {}
    out["fcstYcrps"] = crps_draws(yrealized, ydraws)                                # :358-363
    out["fcstYcumcrps"] = crps_draws(ycumrealized, ycumdraws)                       # :365-370
    out["PAImedian"] = median(PAI_all, 0)                                           # :376
    out["PAImean"] = np.mean(PAI_all, axis=0)                                       # :377
    out["PAIstdev"] = std1(PAI_all, 0)                                              # :378
    out["PAIquantiles"] = np.moveaxis(prctile(PAI_all, pct, 0), 0, 2)               # :379
    out["drawsMaxVARroot"] = max_var_root(PAI_all, N, p)                            # :387-392
    ymed = median(ydraws, 2)
    out["fcstYrealized"] = np.asarray(yrealized, float)
    out["fcstYhat"] = np.asarray(yhat, float)                                       # :451
    out["fcstYmedian"] = ymed
    out["fcstYhaterror"] = yrealized - yhat
    out["fcstYmederror"] = yrealized - ymed
    out["fcstYquantiles"] = np.moveaxis(prctile(ydraws, pct, 2), 0, 2)              # :456
    ymed = median(ycumdraws, 2)
    out["fcstYcumrealized"] = ycumrealized
    out["fcstYcumhat"] = ycumhat
    out["fcstYcummedian"] = ymed
    out["fcstYcumhaterror"] = ycumrealized - ycumhat
    out["fcstYcummederror"] = ycumrealized - ymed
    out["fcstYcumquantiles"] = np.moveaxis(prctile(ycumdraws, pct, 2), 0, 2)        # :466
    out["fcstShadowYhat"] = np.asarray(shadowhat, float)                            # :478
    out["fcstShadowYmedian"] = median(shadowdraws, 2)
    out["fcstShadowYquantiles"] = np.moveaxis(prctile(shadowdraws, pct, 2), 0, 2)   # :480
    return out
