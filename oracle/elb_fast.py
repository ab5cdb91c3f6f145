"""Alternative (exact) formulation of gibbsdrawShadowrates used to design and
cross-check the GPU kernels — TEST INFRASTRUCTURE ONLY.

The reference (gibbsdrawShadowrates.m:74-145) obtains, for every censored month
t, the smoothing weights J_t and the conditional covariance of the shadow rates
S_t by a QR of a 260 x 260 matrix.  They are the moments of the Gaussian
S_t | X_t, past, y_{t+1..t+p} in the zero-mean VAR on Ytilde = Y - Y0.  In a VAR
that conditional factorises exactly:

    p(S_t | ...) ∝ N(y_t; m_t, Λ_t^{-1})|_{X_t fixed} × Π_{k=1..p} N(r_k; B_k S_t, Λ_{t+k}^{-1})

with m_t = Φ s̃_{t-1}, Λ_τ = A' diag(SVol_τ)^{-2} A (A = invA^{-1}), B_k = Φ_k[:, S]
and r_k the lag-k equation residual of y_{t+k} without the S_t term.  Hence

    Ω_t = (Λ_t,SS + Σ_k B_k' Λ_{t+k} B_k)^{-1},
    μ_t(Ỹ) = Ω_t [ (Λ_t m_t)_S − Λ_t,SX Ỹ_X,t + Σ_k B_k' Λ_{t+k} r_k ],
    Spost_t = Y0_S,t + μ_t(Ỹ),

linear in the censored cells of the window: Spost_t = a_t + Σ G S(neighbour).
Per pass that is 3 x 6p multiply-adds per censored month instead of a
240 x 240 matrix-vector product, and the setup is 3 x 3 algebra instead of a
260 x 260 QR.
"""
from __future__ import annotations

import math

import numpy as np

from .ccmm_oracle import draw_trunc_normal


def y0_path(C, STATE0, YHAT0, Ny, T):
    """gibbsdrawShadowrates.m:157-165 (Y0(:,1) = H*STATE0, then advance)."""
    Y0 = np.zeros((Ny, T))
    st0 = np.array(STATE0, dtype=float)
    for t in range(T):
        Y0[:, t] = st0[1:1 + Ny] + (YHAT0[:, t] if YHAT0 is not None else 0.0)
        st0 = C @ st0
    return Y0


def elb_conditionals(Ytil, ndxS, sNaN, p, C, Psi, SVol):
    """For every censored month t: Ω_t (Ns x Ns), the affine map
    Spost_t - Y0_S,t = mu_t(Ytil) as (base, coefficients on censored neighbours)."""
    Ny, T = Ytil.shape
    S = np.flatnonzero(ndxS)
    X = np.flatnonzero(~np.asarray(ndxS))
    Ns = S.size
    Phi = C[1:1 + Ny, 1:]                       # Ny x Ny p
    A = np.linalg.inv(Psi[1:1 + Ny, :])         # invA^{-1}
    Lam = np.einsum("ji,jt,jk->tik", A, 1.0 / SVol ** 2, A)  # T x Ny x Ny

    def mu(t, Yt):
        kmax = min(p, T - 1 - t)
        lag = np.zeros(Ny * p)
        for l in range(1, p + 1):
            if t - l >= 0:
                lag[(l - 1) * Ny:l * Ny] = Yt[:, t - l]
        m = Phi @ lag
        L = Lam[t]
        P = L[np.ix_(S, S)].copy()
        g = (L @ m)[S] - L[np.ix_(S, X)] @ Yt[X, t]
        for k in range(1, kmax + 1):
            Bk = Phi[:, (k - 1) * Ny + S]
            Lk = Lam[t + k]
            r = Yt[:, t + k].copy()
            for l in range(1, p + 1):
                if l == k:
                    r -= Phi[:, (k - 1) * Ny + X] @ Yt[X, t]
                elif t + k - l >= 0:
                    r -= Phi[:, (l - 1) * Ny:l * Ny] @ Yt[:, t + k - l]
            P += Bk.T @ Lk @ Bk
            g += Bk.T @ Lk @ r
        Om = np.linalg.inv(P)
        return Om @ g, Om

    out = {}
    for t in range(T):
        if not sNaN[:, t].any():
            continue
        base, Om = mu(t, Ytil)
        coef = {}
        for tp in range(max(0, t - p), min(T, t + p + 1)):
            if tp == t:
                continue
            for si in range(Ns):
                if sNaN[si, tp]:
                    E = np.zeros_like(Ytil)
                    E[S[si], tp] = 1.0
                    coef[(si, tp)] = mu(t, E)[0]
        out[t] = (base, coef, Om)
    return out


def gibbsdraw_shadowrates_fast(Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, elbBound, Ndraws,
                               burnin, udraws):
    """Same draws as ccmm_oracle.gibbsdraw_shadowrates (to rounding)."""
    ndxS = np.asarray(ndxS, bool)
    Ny, T = Y.shape
    S = np.flatnonzero(ndxS)
    Ns = S.size
    Y0 = y0_path(C, STATE0, YHAT0, Ny, T)
    Scur = Y[S, :].copy()
    Ytil_base = Y - Y0
    Ytil_base[S, :][sNaN] = 0.0
    tmp = Ytil_base[S, :]
    tmp[sNaN] = -Y0[S, :][sNaN]       # censored cells enter with S = 0
    Ytil_base[S, :] = tmp
    cond = elb_conditionals(Ytil_base, ndxS, sNaN, p, C, Psi, SVol)
    draws = np.full((Ns, T, Ndraws), np.nan)
    prec = {}
    for t, (base, coef, Om) in cond.items():
        if Ns > 1:
            b1 = np.zeros((Ns, Ns - 1))
            so = np.zeros(Ns)
            for s in range(Ns):
                o = np.arange(Ns) != s
                b = np.linalg.solve(Om[np.ix_(o, o)].T, Om[s, o])
                b1[s] = b
                so[s] = math.sqrt(Om[s, s] - b @ Om[o, s])
            prec[t] = (b1, so)
        else:
            prec[t] = (None, np.array([math.sqrt(Om[0, 0])]))
    for n in range(burnin + Ndraws):
        for t in sorted(cond):
            base, coef, Om = cond[t]
            Sp = Y0[S, t] + base
            for (si, tp), cvec in coef.items():
                Sp = Sp + cvec * Scur[si, tp]
            b1, so = prec[t]
            if Ns == 1:
                Scur[0, t] = draw_trunc_normal(Sp[0], so[0], elbBound, udraws[0, t, n])[0]
            else:
                for s in np.flatnonzero(sNaN[:, t]):
                    o = np.arange(Ns) != s
                    mu = Sp[s] + b1[s] @ (Scur[o, t] - Sp[o])
                    Scur[s, t] = draw_trunc_normal(mu, so[s], elbBound, udraws[s, t, n])[0]
        if n >= burnin:
            draws[:, :, n - burnin] = Scur
    return draws


# --------------------------------------------------------------------------
# Numerically stable form (what the GPU kernels compute)
# --------------------------------------------------------------------------
# The as-written algorithm forms Ytilde = Y - Y0 and Spost = Y0_S + J Ytilde.  When the
# shadow companion matrix C is explosive (spectral radius > 1 happens for posterior
# draws of PAIshadow), Y0 grows geometrically over the window (1e15 after ~160 months
# at radius 1.2) and both expressions lose every significant digit to cancellation.
# In exact arithmetic Y0 enters only through the lag-equation residuals of its path,
#
#   e0_τ = Y0_τ - Σ_{l<=τ} Φ_l Y0_{τ-l}
#        = [τ = 0: w_{-1};  τ >= 1: c + Σ_{l=τ+1..p} Φ_l w_{τ-1-l}]  +  yhat_τ - Σ_{l<=τ} Φ_l yhat_{τ-l},
#
# (w_{-1-i} = lag block i of STATE0; the recursion w_j = c + Σ Φ_l w_{j-l} cancels the
# rest, including the one-period lag of gibbsdrawShadowrates.m:157-165), which is
# bounded by the data.  With ε_τ(Y) = Y_τ - Σ_{l<=τ} Φ_l Y_{τ-l} - e0_τ the conditional of
# S_t (all Ns rates of month t unknown, neighbours fixed) is
#
#   P S_t = -(Λ_t ε'_t)_S + Σ_k B_k' Λ_{t+k} ε'_{t+k},   ε' = ε evaluated at S_t = 0,
#
# identical to mu_t above in exact arithmetic, with data-scale operands only.

def e0_path(C, STATE0, YHAT0, Ny, T, p):
    Phi = C[1:1 + Ny, 1:]
    c = C[1:1 + Ny, 0]
    X0 = np.asarray(STATE0, float)
    w = lambda i: X0[1 + i * Ny:1 + (i + 1) * Ny]   # w_{-1-i}
    Ph = lambda l: Phi[:, (l - 1) * Ny:l * Ny]
    e0 = np.zeros((Ny, T))
    for t in range(T):
        if t == 0:
            v = w(0).copy()
        else:
            v = c * X0[0]
            for l in range(t + 1, p + 1):
                v = v + Ph(l) @ w(l - t)
        if YHAT0 is not None:
            v = v + YHAT0[:, t]
            for l in range(1, min(p, t) + 1):
                v = v - Ph(l) @ YHAT0[:, t - l]
        e0[:, t] = v
    return e0


def elb_conditionals_stable(Yb, e0, ndxS, sNaN, p, C, Psi, SVol):
    """Per censored month: (a_t, coefficients on censored neighbours, Ω_t) with
    Spost_t = a_t + Σ coef S(neighbour), from the stable residual form."""
    Ny, T = Yb.shape
    S = np.flatnonzero(ndxS)
    Ns = S.size
    Phi = C[1:1 + Ny, 1:]
    A = np.linalg.inv(Psi[1:1 + Ny, :])
    Lam = np.einsum("ji,jt,jk->tik", A, 1.0 / SVol ** 2, A)
    Ph = lambda l: Phi[:, (l - 1) * Ny:l * Ny]

    # base residuals ε_τ(Yb) (censored cells at 0)
    eps = Yb - e0
    for t in range(T):
        for l in range(1, min(p, t) + 1):
            eps[:, t] -= Ph(l) @ Yb[:, t - l]

    cache = {}

    def solve(t, eps_at):
        """eps_at(τ) = residual vector of month τ (t <= τ <= t + kmax).  P_t, Ω_t and the
        products B_k' Λ_{t+k} depend on t only: formed once per month (same operations)."""
        kmax = min(p, T - 1 - t)
        if t not in cache:
            P = Lam[t][np.ix_(S, S)].copy()
            Ms = []
            for k in range(1, kmax + 1):
                Bk = Phi[:, (k - 1) * Ny + S]
                Mk = Bk.T @ Lam[t + k]
                P += Mk @ Bk
                Ms.append(Mk)
            cache.clear()
            cache[t] = (np.linalg.inv(P), Ms)
        Om, Ms = cache[t]
        g = -(Lam[t] @ eps_at(t))[S]
        for k in range(1, kmax + 1):
            g += Ms[k - 1] @ eps_at(t + k)
        return Om @ g, Om

    def unit_eps(q, tp):
        def f(tau):
            v = np.zeros(Ny)
            if tau == tp:
                v[q] = 1.0
            if 1 <= tau - tp <= p:
                v -= Ph(tau - tp)[:, q]
            return v
        return f

    out = {}
    for t in range(T):
        if not sNaN[:, t].any():
            continue
        ySt = Yb[S, t]

        def base_eps(tau, t=t, ySt=ySt):   # ε' : S_t = 0
            v = eps[:, tau].copy()
            if tau == t:
                v[S] -= ySt
            elif 1 <= tau - t <= p:
                v += Phi[:, (tau - t - 1) * Ny + S] @ ySt
            return v

        base, Om = solve(t, base_eps)
        coef = {}
        for tp in range(max(0, t - p), min(T, t + p + 1)):
            if tp == t:
                continue
            for si in range(Ns):
                if sNaN[si, tp]:
                    coef[(si, tp)] = solve(t, unit_eps(S[si], tp))[0]
        out[t] = (base, coef, Om)
    return out


def gibbsdraw_shadowrates_stable(Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, elbBound, Ndraws,
                                 burnin, udraws, return_flags=False):
    """gibbsdrawShadowrates in the stable residual form (same conditionals in exact
    arithmetic; accurate when the shadow companion matrix is explosive).  return_flags: also
    the drawTruncNormal branch flags, Ns x T x (burnin + Ndraws) uint8."""
    ndxS = np.asarray(ndxS, bool)
    Ny, T = Y.shape
    S = np.flatnonzero(ndxS)
    Ns = S.size
    e0 = e0_path(C, STATE0, YHAT0, Ny, T, p)
    Scur = Y[S, :].copy()
    Yb = Y.copy()
    tmp = Yb[S, :]
    tmp[sNaN] = 0.0                                  # censored cells at S = 0
    Yb[S, :] = tmp
    cond = elb_conditionals_stable(Yb, e0, ndxS, sNaN, p, C, Psi, SVol)
    draws = np.full((Ns, T, Ndraws), np.nan)
    flags = np.zeros((Ns, T, burnin + Ndraws), dtype=np.uint8)
    prec = {}
    for t, (base, coef, Om) in cond.items():
        b1 = np.zeros((Ns, max(Ns - 1, 0)))
        so = np.zeros(Ns)
        for s in range(Ns):
            o = np.arange(Ns) != s
            if Ns > 1:
                b1[s] = np.linalg.solve(Om[np.ix_(o, o)].T, Om[s, o])
                so[s] = math.sqrt(Om[s, s] - b1[s] @ Om[o, s])
            else:
                so[s] = math.sqrt(Om[0, 0])
        prec[t] = (b1, so)
    for n in range(burnin + Ndraws):
        for t in sorted(cond):
            base, coef, Om = cond[t]
            Sp = base.copy()
            for (si, tp), cvec in coef.items():
                Sp = Sp + cvec * Scur[si, tp]
            b1, so = prec[t]
            for s in np.flatnonzero(sNaN[:, t]):
                o = np.arange(Ns) != s
                mu = Sp[s] + (b1[s] @ (Scur[o, t] - Sp[o]) if Ns > 1 else 0.0)
                Scur[s, t], flags[s, t, n] = draw_trunc_normal(mu, so[s], elbBound, udraws[s, t, n])
        if n >= burnin:
            draws[:, :, n - burnin] = Scur
    return (draws, flags) if return_flags else draws
