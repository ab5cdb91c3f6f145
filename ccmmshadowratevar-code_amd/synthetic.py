"""Synthetic data of the S120 stress configuration (BASELINE.json configs[4]; SURVEY.md
§8d C5): a block-hybrid shadow-rate VAR panel with N = 120 series, p = 12 lags and
T = 750 months after a 12-month presample (K = N p + 1 = 1441).

The reference has no such data set: its CSVs hold N = 20 series.  The generator follows
SURVEY §8d C5: Pi_1 = 0.5 I plus U(-0.02, 0.02) off-diagonals, Pi_l = (0.3 / l^2) I for
l >= 2, rescaled until the companion spectral radius is <= 0.95; A unit lower with
N(0, 0.1^2) below the diagonal; log h random walks with sigma 0.05 from 0; six "yield"
series are persistent AR(1) levels that sit below the 0.25 ELB for their last ~15 % of
months.  The yields carry the reference's names (setShadowYields.m): FEDFUNDS, TB3MS,
TB6MS and GS1 are the shadow rates, GS5 and GS10 the other yields.
"""
from __future__ import annotations

import datetime

import numpy as np

SEED = 20230101
YIELD_NAMES = ("FEDFUNDS", "TB3MS", "TB6MS", "GS1", "GS5", "GS10")


def _spectral_radius(Pi, N, p):
    comp = np.zeros((N * p, N * p))
    comp[:N, :] = np.hstack(Pi)
    comp[N:, :N * (p - 1)] = np.eye(N * (p - 1))
    return float(np.max(np.abs(np.linalg.eigvals(comp))))


def s120(N=120, p=12, T=750, seed=SEED, elb=0.25, elb_share=0.15):
    """Returns dict(data (T+p) x N, ydates (monthly MATLAB datenums), ncode, p, elb)."""
    rng = np.random.default_rng(seed)
    Pi = [0.5 * np.eye(N) + rng.uniform(-0.02, 0.02, (N, N)) * (1 - np.eye(N))]
    Pi += [(0.3 / l ** 2) * np.eye(N) for l in range(2, p + 1)]
    rho = _spectral_radius(Pi, N, p)
    while rho > 0.95:
        Pi = [P * (0.95 / rho) ** (1.0 / (l + 1)) for l, P in enumerate(Pi)]
        rho = _spectral_radius(Pi, N, p)
    A = np.eye(N) + np.tril(rng.normal(0.0, 0.1, (N, N)), -1)
    invA = np.linalg.solve(A, np.eye(N))
    Tobs = T + p
    y = np.zeros((Tobs, N))
    y[:p] = rng.standard_normal((p, N))
    lh = np.zeros(N)
    c = 0.1 * rng.standard_normal(N)
    for t in range(p, Tobs):
        lh = lh + 0.05 * rng.standard_normal(N)
        y[t] = c + sum(Pi[l] @ y[t - 1 - l] for l in range(p)) + invA @ (np.exp(lh / 2) * rng.standard_normal(N))
    # six yields: persistent AR(1) levels, below the ELB over the last ~15 % of months
    ny = len(YIELD_NAMES)
    ycols = np.arange(N - ny, N)
    t_elb = int(round(Tobs * (1 - elb_share)))
    for k, col in enumerate(ycols):
        lev = np.empty(Tobs)
        lev[0] = 4.0 + 0.5 * k
        for t in range(1, Tobs):
            lev[t] = 0.2 + 0.985 * (lev[t - 1] - 0.2) + 0.2 * rng.standard_normal()
        lev[:t_elb] = np.abs(lev[:t_elb] - elb) + elb + 0.05 + 0.1 * k   # above the ELB before
        lev[t_elb:] = elb - rng.uniform(0.02, 0.2, Tobs - t_elb)        # at the ELB after
        y[:, col] = lev
    d0 = datetime.date(1959, 3, 1)
    ydates = []
    for t in range(Tobs):
        yy, mm = d0.year + (d0.month - 1 + t) // 12, (d0.month - 1 + t) % 12 + 1
        ydates.append(float(datetime.date(yy, mm, 1).toordinal() + 366))
    ncode = [f"X{i:03d}" for i in range(N - ny)] + list(YIELD_NAMES)
    return dict(data=y, ydates=np.array(ydates), ncode=ncode, p=p, elb=elb)
