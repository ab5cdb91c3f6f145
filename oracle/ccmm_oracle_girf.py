"""Oracle (CPU restatement) of the generalized impulse responses of generateGIRF2linear.m /
generateGIRF2blockhybrid.m — TEST INFRASTRUCTURE ONLY (device path: ccmm_girf.hip).

Per MCMC draw mm (generateGIRF2blockhybrid.m:199-259): SV paths
SVdraws = exp(cumsum(chol(PHI,'lower') * randn(N, H*nsim), 2) / 2), and antitheticSim
(:394-425): four shock sets z .* SV .* SV0, -z .* SV .* SV0, z ./ SV .* SV0, -z ./ SV .* SV0
(SV0 = the jump-off sqrtht), each with shock11 added to element (1, 1); simVAR* maps the
shocks through invA and simulates the companion system (linear: ltitr, :369-382 of the
linear file; block hybrid: actual-rate states max(shadow, ELB) and yields floored at the
ELB, :369-391); cumcode variables cumsum / np; the mean over the 4 nsim paths.  Returns the
baseline, +shock and -shock mean paths (fcstYHATdraws, ...1plus, ...1minus)."""
from __future__ import annotations

import numpy as np


def companion_hybrid(PAI, N, p, shadow):
    """fcstA of generateGIRF2hybrid.m:178-185, 226-227: Nstates = K + p Ns, the companion rows
    are the hybrid PAI itself ((K + Ns p) x N), a shift for the Ns actual-rate lags."""
    K = 1 + N * p
    Ns = int(np.count_nonzero(shadow))
    ns = K + p * Ns
    A = np.zeros((ns, ns))
    A[0, 0] = 1.0
    A[1 + N:K, 1:K - N] = np.eye(N * (p - 1))
    A[K + Ns:, K:ns - Ns] = np.eye(Ns * (p - 1))
    A[1:1 + N, :] = PAI.T
    return A


def companion(PAI, N, p, bh=False, actual=None, yields=None):
    """fcstA (generateGIRF2blockhybrid.m:183-189, 226-234): K states [1, y lags] and for the
    block hybrid p blocks of the Ny actual-rate lags."""
    K = 1 + N * p
    if not bh:
        A = np.zeros((K, K))
        A[0, 0] = 1.0
        A[1 + N:, 1:K - N] = np.eye(N * (p - 1))
        A[1:1 + N, :] = PAI.T
        return A
    yidx = np.flatnonzero(yields)
    Ny = yidx.size
    ns = K + p * Ny
    A = np.zeros((ns, ns))
    A[0, 0] = 1.0
    A[1 + N:K, 1:K - N] = np.eye(N * (p - 1))
    A[K + Ny:, K:ns - Ny] = np.eye(Ny * (p - 1))
    lagY = np.concatenate([[False], np.tile(np.asarray(yields, bool), p)])
    PAIactual = PAI[lagY, :].T.copy()                 # N x (p Ny)
    PAIactual[~np.asarray(actual, bool), :] = 0.0
    PAIshadow = PAI.T.copy()
    PAIshadow[np.ix_(np.asarray(actual, bool), lagY)] = 0.0
    A[1:1 + N, :K] = PAIshadow
    A[1:1 + N, K:] = PAIactual
    return A


def girf_draw(PAI, invA, sqrtPHI, SV0, Xjumpoff, z, svz, shock11, cumcode, np_, bh=False,
              actual=None, yields=None, elb=0.25, shadow=None, p=None):
    """One MCMC draw.  z, svz: N x H x nsim (zdraws; fcstSVdraws reshaped).  Returns
    (yhat_base, yhat_plus, yhat_minus), each N x H.  shadow (N bools) selects the hybrid model
    (generateGIRF2hybrid.m, simVARhybrid :361-386): PAI (K + Ns p) x N, the actual-rate ring
    holds the shadow-rate variables, the output floors ``yields``."""
    N, H, nsim = z.shape
    hybrid = shadow is not None
    if hybrid:
        Ns = int(np.count_nonzero(shadow))
        p = (PAI.shape[0] - 1) // (N + Ns) if p is None else p
        A = companion_hybrid(PAI, N, p, shadow)
        ring = np.flatnonzero(shadow)
        bh = True
    else:
        p = (PAI.shape[0] - 1) // N
        A = companion(PAI, N, p, bh, actual, yields)
        ring = np.flatnonzero(yields) if bh else np.array([], int)
    ns = A.shape[0]
    yidx = np.flatnonzero(yields) if bh else np.array([], int)
    K = 1 + N * p
    SV = np.exp(np.cumsum(np.einsum("ij,jhn->ihn", sqrtPHI, svz), axis=1) * 0.5)
    cc = np.asarray(cumcode, bool)

    def sim(nu):                                   # nu: N x H x nsim
        out = np.empty((N, H, nsim))
        for nn in range(nsim):
            sh = invA @ nu[:, :, nn]
            x = np.array(Xjumpoff, float)
            for h in range(H):
                xn = A @ x
                xn[1:1 + N] += sh[:, h]
                out[:, h, nn] = xn[1:1 + N]
                x = xn
                if bh:
                    x[K:K + ring.size] = np.maximum(x[1 + ring], elb)
        if bh:
            yy = out[yidx]
            yy[yy < elb] = elb
            out[yidx] = yy
        out[cc] = np.cumsum(out[cc], axis=1) / np_
        return out

    res = []
    for s11 in (0.0, shock11, -shock11):
        ys = []
        for sz, up in ((1, True), (-1, True), (1, False), (-1, False)):
            nu = sz * z * (SV if up else 1.0 / SV) * SV0[:, None, None]
            nu[0, 0, :] += s11
            ys.append(sim(nu))
        res.append(np.mean(np.concatenate(ys, axis=2), axis=2))
    return tuple(res)
