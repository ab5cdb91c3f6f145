"""CPU checks of the GIRF oracle (oracle/ccmm_oracle_girf.py): the antithetic mean of the
linear simulation is the deterministic path (the shocks cancel pairwise), so +shock minus
baseline equals the impulse response; the block-hybrid companion reproduces the linear
one when no equation is in the actual-rate block and the ELB never binds."""
import numpy as np


def _draw(rng, N, p):
    K = 1 + N * p
    PAI = 0.05 * rng.standard_normal((K, N))
    PAI[1:1 + N] += 0.5 * np.eye(N)
    invA = np.eye(N) + np.tril(0.2 * rng.standard_normal((N, N)), -1)
    sqrtPHI = np.diag(0.05 + 0.1 * rng.random(N))
    return PAI, invA, sqrtPHI


def test_linear_girf_is_irf():
    from oracle import ccmm_oracle_girf as gi
    rng = np.random.default_rng(1)
    N, p, H, nsim = 4, 2, 6, 5
    PAI, invA, sqrtPHI = _draw(rng, N, p)
    Xj = np.r_[1.0, rng.standard_normal(N * p)]
    z, svz = rng.standard_normal((2, N, H, nsim))
    b, pl, mi = gi.girf_draw(PAI, invA, sqrtPHI, 0.5 + rng.random(N), Xj, z, svz, 0.5,
                             np.zeros(N, bool), 12)
    A = gi.companion(PAI, N, p)
    x = np.zeros(A.shape[0])
    x[1:1 + N] = invA[:, 0] * 0.5
    irf = []
    for _ in range(H):
        irf.append(x[1:1 + N].copy())
        x = A @ x
    irf = np.array(irf).T
    assert np.max(np.abs(pl - b - irf)) < 1e-13 and np.max(np.abs(b - mi - irf)) < 1e-13


def test_bh_companion_without_actual_block_is_linear():
    from oracle import ccmm_oracle_girf as gi
    rng = np.random.default_rng(2)
    N, p, H, nsim = 4, 2, 5, 3
    PAI, invA, sqrtPHI = _draw(rng, N, p)
    yields = np.array([False, True, False, True])
    Xj = np.r_[1.0, 5 + rng.random(N * p)]
    Xbh = np.r_[Xj, 5 + rng.random(2 * p)]
    z, svz = 0.1 * rng.standard_normal((2, N, H, nsim))
    SV0 = 0.5 + rng.random(N)
    lin = gi.girf_draw(PAI, invA, sqrtPHI, SV0, Xj, z, svz, 0.3, np.zeros(N, bool), 12)
    bh = gi.girf_draw(PAI, invA, sqrtPHI, SV0, Xbh, z, svz, 0.3, np.zeros(N, bool), 12, bh=True,
                      actual=np.zeros(N, bool), yields=yields, elb=-100.0)
    for a, b in zip(lin, bh):
        assert np.max(np.abs(a - b)) < 1e-12
