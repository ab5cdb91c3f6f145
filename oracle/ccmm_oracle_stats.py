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
