"""Test infrastructure (CPU oracle): Geweke's numerical standard errors as the reference
computes them (Diagnostics.m:134-300, ``momentg``), used by the Monte Carlo standard-error
(MCSE) parity test of the Philox chains.  Not part of the product path.

momentg groups the first nuse = NG * floor(ndraw / NG) draws into NG = 100 consecutive
groups.  With the weights ad = 1 of Diagnostics.m:199 the sufficient statistics reduce to
(per variable, g the draws):
  pmean = mean(g),  pstd = sqrt(mean(g^2) - pmean^2)                       (:219-224)
  nse   = sqrt(sum (g - pmean)^2) / nuse                                   (:229-231)
  r(l)  = sum_{ig > l} cbar_ig cbar_{ig-l} / NG,  cbar = group means - pmean (:238-252)
  nse_m = sqrt(ns / nuse * (r(0) + 2 sum_{l=1}^{m-1} (1 - l/m) r(l))),  m = 4, 8, 15 (:256-266)
  rne*  = pstd^2 / (nuse * nse*^2)
"""
from __future__ import annotations

import numpy as np

NG = 100
TAPERS = (4, 8, 15)


def momentg(draws):
    """draws: ndraw x nvar.  Returns a dict of nvar-vectors (Diagnostics.m:134-300)."""
    draws = np.asarray(draws, dtype=float)
    if draws.ndim == 1:
        draws = draws[:, None]
    ndraw, nvar = draws.shape
    if ndraw < NG:
        raise ValueError("momentg: needs a larger number of ndraws")
    ns = ndraw // NG
    nuse = ns * NG
    g = draws[:nuse]
    eg = g.mean(axis=0)
    varg = (g * g).mean(axis=0) - eg ** 2
    out = {"ndraw": ndraw, "nvar": nvar, "pmean": eg,
           "pstd": np.where(varg > 0, np.sqrt(np.maximum(varg, 0.0)), -1.0)}
    varnum = ((g - eg) ** 2).sum(axis=0) / nuse ** 2
    out["nse"] = np.where(varnum > 0, np.sqrt(np.maximum(varnum, 0.0)), -1.0)
    out["rne"] = varg / (nuse * varnum)
    cn = g.reshape(NG, ns, nvar).mean(axis=1) - eg          # grouped means - pmean
    rnn = np.array([(cn[lag:] * cn[:NG - lag]).sum(axis=0) / NG for lag in range(NG)])
    for k, m in enumerate(TAPERS, start=1):
        snn = rnn[0] + 2.0 * sum((1.0 - lag / m) * rnn[lag] for lag in range(1, m))
        vn = ns * snn / nuse
        out[f"nse{k}"] = np.where(vn > 0, np.sqrt(np.maximum(vn, 0.0)), -1.0)
        out[f"rne{k}"] = varg / (nuse * vn)
    return out


def psrf(X):
    """Potential scale reduction factor as DiagnosticsShadowrate.m:34-134 computes it
    (Brooks & Gelman 1998, square-root form; the same function as Diagnostics.m:28).

    X: n x D (one chain: split into its first and last thirds, :82-91) or n x D x M
    (M sequences).  Statement order of :106-128: W = sum_i sum_t (x - mean_i)^2 / ((n-1) M),
    Bpn = sum_i (mean_i - m)^2 / (M - 1), S = (n-1)/n W + Bpn,
    R = sqrt((M+1)/M S / W - (n-1)/M/n).  Returns R (D,)."""
    X = np.asarray(X, dtype=float)
    if X.ndim == 1:
        X = X[:, None]
    if X.ndim == 2:
        n = X.shape[0] // 3                                  # floor(size(X,1)/3), :85
        X = np.stack([X[:n], X[X.shape[0] - n:]], axis=2)    # first and last thirds, :87-88
    n, D, M = X.shape
    if n < 1:
        raise ValueError("Too few samples")                  # :103-105
    W = np.zeros(D)
    for i in range(M):                                       # :108-113
        x = X[:, :, i] - X[:, :, i].mean(axis=0)
        W = W + (x * x).sum(axis=0)
    W = W / ((n - 1) * M)
    means = X.mean(axis=0)                                   # D x M
    m = means.mean(axis=1)                                   # :117
    Bpn = np.zeros(D)
    for i in range(M):                                       # :118-122
        x = means[:, i] - m
        Bpn = Bpn + x * x
    Bpn = Bpn / (M - 1)
    S = (n - 1) / n * W + Bpn                                # :125-128
    with np.errstate(divide="ignore", invalid="ignore"):
        R = (M + 1) / M * S / W - (n - 1) / M / n
        return np.sqrt(R)


def diagnostics_shadowrate(draws):
    """DiagnosticsShadowrate.m:1-22: mean over the shadow-rate cells of psrf(draws), draws
    n x nObs (n x nObs x M for M chains); NaN when there are no cells (mean of an empty row)."""
    draws = np.asarray(draws, dtype=float)
    if draws.shape[1] == 0:
        return float("nan")
    return float(np.mean(psrf(draws)))


def diagnostics_shadowrate_chain_mean(draws):
    """DiagnosticsShadowrate (one-chain form: first / last thirds) of each of the C chains of draws
    n x nObs x C, averaged over the chains: the reference's statistic for a multi-chain run."""
    draws = np.asarray(draws, dtype=float)
    return float(np.mean([diagnostics_shadowrate(draws[:, :, c]) for c in range(draws.shape[2])]))
