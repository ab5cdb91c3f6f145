#!/usr/bin/env python
"""Developer check: the partitioned SV sampler (oracle.sv_draw_partitioned) has the
exact posterior moments — mean P^{-1} b and covariance P^{-1} — for several
(N, T), by building the dense precision and the draw's linear map in z."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import ccmm_oracle as O  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    for N, T in [(3, 20), (4, 60), (2, 7), (5, 130), (2, 3)]:
        obs = rng.standard_normal((N, T))
        ir = rng.uniform(0.5, 3, (N, T))
        L = np.tril(rng.uniform(-0.1, 0.1, (N, N)), -1) + np.diag(rng.uniform(0.1, 0.3, N))
        D, b, Q = O.sv_precision(obs, ir, L, np.zeros(N), 10 * np.eye(N))
        T1 = T + 1
        P = np.zeros((T1 * N, T1 * N))
        for t in range(T1):
            P[t * N:(t + 1) * N, t * N:(t + 1) * N] = D[t]
            if t:
                P[t * N:(t + 1) * N, (t - 1) * N:t * N] = -Q
                P[(t - 1) * N:t * N, t * N:(t + 1) * N] = -Q
        mean = np.linalg.solve(P, b.ravel())
        z0 = np.zeros((N, T1))
        xp = O.sv_draw_partitioned(D, b, Q, z0)
        xs = O.sv_draw_sequential(D, b, Q, z0)
        M = np.zeros((T1 * N, T1 * N))
        for j in range(T1 * N):
            z = np.zeros(T1 * N)
            z[j] = 1
            M[:, j] = O.sv_draw_partitioned(D, b, Q, z.reshape(T1, N).T).ravel() - xp.ravel()
        Pi = np.linalg.inv(P)
        print(N, T, len(O.sv_separators(T)), "mean", np.abs(xp.ravel() - mean).max(),
              np.abs(xs.ravel() - mean).max(), "cov", np.abs(M @ M.T - Pi).max() / np.abs(Pi).max())


if __name__ == "__main__":
    main()
