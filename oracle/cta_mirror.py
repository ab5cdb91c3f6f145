"""CTA in the device's operation order -- TEST INFRASTRUCTURE ONLY (the checker of
tests/test_gpu_mirror.py; never imported by the product).

ccmm_oracle.cta / cta_syrk restate CTA.m:57-98 (as written / algorithmic); at the conditioning
of the real data (cond(iV_post) ~ 1e9 with smooth volatility) a mere change of summation order
moves a draw by ~1e-8 posterior sd, so those forms cannot pin the device to the
1e-9 of the north star.  This form evaluates the same posterior with the device's weights,
weighted Gram (v_mfma_f64_16x16x4_f64: fused multiply-adds in k order, measured by
tools/probe_mfma_order.py), residuals, right-hand side, intercept peel, tiled right-looking
Cholesky with 16 x 16 diagonal-tile inverses, and the block substitutions of the unit block
factor, operation for operation (oracle/cta_lag_mirror.c; ccmm_lag.hip).  factor="lapack" keeps
the previous form (LAPACK Cholesky and triangular solves of the mirrored Gram) for comparison.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
from scipy.linalg import cholesky, solve_triangular

_HERE = Path(__file__).resolve().parent
_LIB = None
_dp = C.POINTER(C.c_double)


def lib():
    global _LIB
    if _LIB is None:
        so = _HERE / "libccmm_mirror.so"
        srcs = [_HERE / "cta_lag_mirror.c", _HERE / "cta_big_mirror.c"]
        if not so.exists() or so.stat().st_mtime < max(f.stat().st_mtime for f in srcs):
            subprocess.run(["make", "-C", str(_HERE)], check=True, capture_output=True)
        _LIB = C.CDLL(str(so))
        for name, args in (("ccmm_mirror_weights", [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp]),
                           ("ccmm_mirror_gram", [C.c_int, C.c_int, _dp, _dp, _dp]),
                           ("ccmm_mirror_resid", [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp]),
                           ("ccmm_mirror_v", [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp]),
                           ("ccmm_mirror_rhs", [C.c_int, C.c_int, _dp, _dp, _dp, _dp]),
                           ("ccmm_mirror_resid_update", [C.c_int, C.c_int, _dp, _dp, _dp, _dp]),
                           ("ccmm_mirror_solve", [C.c_int, _dp, _dp, C.c_double, _dp, _dp, _dp])):
            f = getattr(_LIB, name)
            f.argtypes = args
            f.restype = None
        _LIB.ccmm_mirror_factor.argtypes = [C.c_int, _dp, _dp, _dp, _dp, _dp]
        _LIB.ccmm_mirror_factor.restype = C.c_int
        _LIB.ccmm_bmirror_cta.argtypes = [C.c_int, C.c_int, C.c_int] + [_dp] * 9
        _LIB.ccmm_bmirror_cta.restype = C.c_int
    return _LIB


def _p(a):
    return a.ctypes.data_as(_dp)


def _F(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def weights(A, sqrtht, j):
    T, N = sqrtht.shape
    sw = np.zeros(T)
    A, sh = _F(A), _F(sqrtht)
    lib().ccmm_mirror_weights(T, N, j, _p(A), _p(sh), _p(sw))
    return sw


def gram(X, sw):
    """[c b'; b M] of the device SYRK stage (no prior), K x K."""
    T, K = X.shape
    X = _F(X)
    G = np.zeros((K, K), order="F")
    lib().ccmm_mirror_gram(T, K, _p(X), _p(np.ascontiguousarray(sw)), _p(G))
    return G


def factor(G, iv):
    """Device-order factorisation of G + diag(iv) (G = [c b'; b M] from gram()): returns the
    factor record (slots, l, 1 / L00) and the non-positive-pivot flag."""
    K = G.shape[0]
    NT = (K - 1 + 15) // 16
    S = np.zeros(NT * NT * 256)
    lv = np.zeros(16 * NT)
    r = C.c_double(0.0)
    bad = lib().ccmm_mirror_factor(K, _p(_F(G)), _p(np.ascontiguousarray(iv, dtype=np.float64)), _p(S), _p(lv),
                                   C.byref(r))
    return (S, lv, r.value), bool(bad)


def solve(fac, rhs, z):
    """x = L' \\ (L \\ rhs + z) in the device's substitution order."""
    S, lv, rL00 = fac
    K = rhs.size
    x = np.zeros(K)
    lib().ccmm_mirror_solve(K, _p(S), _p(lv), rL00, _p(np.ascontiguousarray(rhs, dtype=np.float64)),
                            _p(np.ascontiguousarray(z, dtype=np.float64)), _p(x))
    return x


def cta(Y, X, N, K, A, sqrtht, iVdiag, iVb, PAI, z, factor_form="device"):
    """CTA.m:57-98 (CTA: one design) with the device's arithmetic throughout (factor_form="lapack":
    LAPACK Cholesky and solves of the mirrored Gram and right-hand side).  X may also be a list of
    N per-equation designs: CTAsys.m:57-108 (the block hybrid's actual-rate and shadow-rate slabs,
    mcmcVARshadowrateBlockHybrid.m:341), each equation's Gram, right-hand side and residual on its
    own design, in the same device order."""
    T = Y.shape[0]
    Y, A, sh = _F(Y), _F(A), _F(sqrtht)
    Xs = [_F(x) for x in X] if isinstance(X, (list, tuple)) else [_F(X)] * N
    PAI = _F(PAI).copy(order="F")
    E = np.zeros((T, N), order="F")
    L_ = lib()
    for j in range(N):                   # one residual column per equation, on its own design
        Ej = np.zeros(T)
        L_.ccmm_mirror_resid(T, K, 1, _p(np.ascontiguousarray(Y[:, j])), _p(Xs[j]),
                             _p(np.ascontiguousarray(PAI[:, j])), _p(Ej))
        E[:, j] = Ej
    v = np.zeros(T)
    rhs = np.zeros(K)
    for j in range(N):
        X = Xs[j]
        sw = weights(A, sh, j)
        G = gram(X, sw)
        L_.ccmm_mirror_v(T, N, j, _p(A), _p(sh), _p(Y), _p(E), _p(v))
        ivb = np.ascontiguousarray(iVb[:, j], dtype=np.float64)
        L_.ccmm_mirror_rhs(T, K, _p(X), _p(v), _p(ivb), _p(rhs))
        if factor_form == "lapack":
            Gp = G.copy()
            Gp[np.diag_indices(K)] += iVdiag[:, j]
            Lc = cholesky(Gp, lower=True)
            x = solve_triangular(Lc.T, solve_triangular(Lc, rhs, lower=True) + z[:, j], lower=False)
        else:
            fac, _ = factor(G, iVdiag[:, j])
            x = solve(fac, rhs, z[:, j])
        PAI[:, j] = x
        xj = np.ascontiguousarray(x)
        Ej = np.zeros(T)
        L_.ccmm_mirror_resid_update(T, K, _p(X), _p(np.ascontiguousarray(Y[:, j])), _p(xj), _p(Ej))
        E[:, j] = Ej
    return np.array(PAI)


def cta_big(Y, X, N, K, A, sqrtht, iVdiag, iVb, PAI, z):
    """CTA.m:57-98 through the device's large-system path (ccmm_big.hip: k_gram_big, k_chol_big,
    k_cta_solve_big; oracle/cta_big_mirror.c) in its operation order: the hybrid model's
    K = 1 + (N + Ns) p design (mcmcVARhybridGibbs.m:74-84) and every system off the lag path.
    Returns (PAI, bad) with bad = 1 for a non-positive pivot."""
    T = Y.shape[0]
    out = np.zeros((K, N), order="F")
    bad = lib().ccmm_bmirror_cta(T, N, K, _p(_F(Y)), _p(_F(X)), _p(_F(A)), _p(_F(sqrtht)), _p(_F(iVdiag)),
                                 _p(_F(iVb)), _p(_F(PAI)), _p(_F(z)), _p(out))
    return np.array(out), int(bad)
