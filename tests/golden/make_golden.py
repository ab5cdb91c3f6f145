"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference (MATLAB) cannot run in this image and ships no fixtures
(SURVEY.md §8c), so these vectors are produced by this build's restatement
(oracle/ccmm_oracle.py) and, where the fp64 answer is ill-conditioned, by an
80-bit long-double evaluation of the same algebra.  Run from the repo root:

    python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle import ccmm_oracle as O  # noqa: E402
from helpers import crn_flat, random_state, toy_setup  # noqa: E402

OUT = Path(__file__).resolve().parent
CSV = OUT / "data" / "fredblockMD20-2022-09.csv"


def cta_syrk_longdouble(su, st, z):
    """CTA (weighted-SYRK form, Cholesky + triangular solves) in np.longdouble."""
    dt = np.longdouble
    Y, X = su.Y.astype(dt), su.X.astype(dt)
    A, sh = st["A"].astype(dt), st["sqrtht"].astype(dt)
    PAI = st["PAI"].astype(dt).copy()
    N, K = su.N, su.K
    for j in range(N):
        PAI[:, j] = 0
        E = Y - X @ PAI
        ih2 = 1 / sh[:, j:] ** 2
        w = ih2 @ (A[j:, j] ** 2)
        v = ((E @ A[j:, :].T) * ih2) @ A[j:, j]
        P = np.diag(su.iVdiag[:, j].astype(dt)) + X.T @ (X * w[:, None])
        rhs = su.iVb[:, j].astype(dt) + X.T @ v
        L = np.zeros_like(P)
        for k in range(K):
            L[k, k] = np.sqrt(P[k, k] - L[k, :k] @ L[k, :k])
            L[k + 1:, k] = (P[k + 1:, k] - L[k + 1:, :k] @ L[k, :k]) / L[k, k]
        y = np.zeros(K, dt)
        for k in range(K):
            y[k] = (rhs[k] - L[k, :k] @ y[:k]) / L[k, k]
        y = y + z[:, j].astype(dt)
        x = np.zeros(K, dt)
        for k in range(K - 1, -1, -1):
            x[k] = (y[k] - L[k + 1:, k] @ x[k + 1:]) / L[k, k]
        PAI[:, j] = x
    return PAI.astype(float)


def main():
    fred = O.load_fred_csv(CSV)
    mpm = O.set_minnesota_mean(fred["ncode"])
    su = O.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)

    # (ii) real-data CTA at the reference initialisation (mcmcVAR.m:197-206), z = seed 5
    st = O.init_state(su)
    z = np.random.default_rng(5).standard_normal((su.K, su.N))
    pai_o, _, sd = O.cta(su.Y, su.X, su.N, su.K, st["A"], st["sqrtht"], su.iVdiag, su.iVb,
                         st["PAI"], z, return_sd=True)
    pai_ld = cta_syrk_longdouble(su, st, z)
    np.savez_compressed(OUT / "cta_refinit.npz", z=z, PAI_oracle=pai_o, PAI_longdouble=pai_ld,
                        sd=sd)

    # (i) toy N=4, p=2, T=60: three CRN sweeps from a perturbed state
    tsu = toy_setup(O, N=4, p=2, Tobs=62, seed=0)
    tst = random_state(O, tsu, seed=1)
    rng = np.random.default_rng(2024)
    crns = [O.draw_crn(rng, tsu.N, tsu.K, tsu.T, tsu.dPHI) for _ in range(3)]
    s = tst
    outs = {}
    for m, crn in enumerate(crns):
        s = O.linear_sweep(s, tsu, crn)
        for k in ("PAI", "A", "invA", "sqrtht", "h", "sqrtPHI", "PHI", "kai"):
            outs[f"sweep{m}_{k}"] = s[k]
    np.savez_compressed(OUT / "toy_linear_sweeps.npz",
                        data=tsu.data,
                        Y=tsu.Y, X=tsu.X, iVdiag=tsu.iVdiag, iVb=tsu.iVb, sPHI=tsu.sPHI,
                        state_PAI=tst["PAI"], state_A=tst["A"], state_sqrtht=tst["sqrtht"],
                        state_h=tst["h"], state_sqrtPHI=tst["sqrtPHI"],
                        crn=np.stack([crn_flat(O, c, tsu) for c in crns], -1), **outs)

    # (iii) truncated-normal known answers incl. both degenerate branches
    rng = np.random.default_rng(77)
    mu = np.concatenate([rng.normal(0.5, 2.0, 200), [40.0, 60.0, 0.1, -3.0], [0.2] * 4])
    sig = np.concatenate([np.abs(rng.normal(0, 1, 200)), [1.0, 2.0, 1e-12, 0.0],
                          [0.5, 0.5, 0.5, 0.5]])
    u = np.concatenate([rng.random(204), [1e-300, 1e-12, 0.5, 1 - 1e-16]])
    res = np.array([O.draw_trunc_normal(mu[i], sig[i], 0.25, u[i]) for i in range(mu.size)])
    np.savez_compressed(OUT / "truncnorm_kat.npz", mu=mu, sig=sig, u=u, elb=0.25,
                        draw=res[:, 0], flags=res[:, 1].astype(np.uint8))

    # (iv) KSC indicator vectors
    rng = np.random.default_rng(99)
    y = rng.normal(-1.0, 3.0, (6, 50))
    hp = rng.normal(0.0, 1.0, (6, 50))
    u = rng.random((6, 50))
    np.savez_compressed(OUT / "ksc_indicators.npz", y=y, h=hp, u=u,
                        kai=O.ksc_indicators(y, hp, u))
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
