"""Shared inputs for the predictive-density tests (mcmcVAR.m:298-381): a real-data
kept draw (fredblockMD20-2022-09.csv, N=20, p=12, K=241) with yields at the ELB in
0, 1, 2 or 3 positions of the realized vector."""
import numpy as np


def fcst_inputs(oracle, fred, B=4, H=48, Nd=10, seed=11, nat=(0, 1, 2, 3)):
    data = fred["data"]
    N, p = data.shape[1], 12
    K = N * p + 1
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    yields = np.zeros(N, bool)
    yields[np.concatenate([ndxS, ndxO])] = True
    rng = np.random.default_rng(seed)
    # OLS coefficients at the last vintage (the reference initialisation PAI = X\Y)
    X = np.hstack([np.ones((len(data) - p, 1))] + [data[p - l:len(data) - l] for l in range(1, p + 1)])
    Y = data[p:]
    PAI0 = np.linalg.lstsq(X, Y, rcond=None)[0]
    Xj = np.concatenate([[1.0]] + [data[len(data) - 1 - l] for l in range(p)])
    PAI = np.empty((K, N, B)); invA = np.empty((N, N, B)); logSV0 = np.empty((N, B))
    sqrtPHI = np.empty((N, N, B)); Xjs = np.empty((K, B))
    resid_var = np.var(Y - X @ PAI0, axis=0)
    # an arbitrary kept draw whose shadow-rate means sit just above the ELB (intercept shift)
    PAI0 = PAI0.copy()
    PAI0[0, ndxS] -= PAI0[:, ndxS].T @ Xj - 0.35
    for c in range(B):
        PAI[:, :, c] = PAI0 + 1e-3 * rng.standard_normal((K, N))
        A = np.eye(N) + np.tril(rng.uniform(-0.4, 0.4, (N, N)), -1)
        invA[:, :, c] = np.linalg.solve(A, np.eye(N))
        logSV0[:, c] = np.log(resid_var) + 0.2 * rng.standard_normal(N)
        sqrtPHI[:, :, c] = np.tril(rng.uniform(-0.02, 0.02, (N, N)), -1) + np.diag(rng.uniform(0.05, 0.15, N))
        Xjs[:, c] = Xj
    svz = rng.standard_normal((N, H * Nd, B))
    z = rng.standard_normal((N, H, Nd, B))
    # realized values: the one-step mean plus noise; put `n` shadow-rate yields at the ELB
    ys = []
    for n in nat:
        y = PAI0.T @ Xj + 0.1 * rng.standard_normal(N)
        y[yields] = np.maximum(y[yields], 0.45)
        at = np.concatenate([ndxS, ndxO])[:n]
        y[at] = 0.25 - rng.uniform(0.0, 0.15, n)
        ys.append(y)
    return dict(PAI=PAI, invA=invA, logSV0=logSV0, sqrtPHI=sqrtPHI, Xj=Xjs, yields=yields,
                svz=svz, z=z, ys=ys, H=H, Nd=Nd, elb=0.25)
