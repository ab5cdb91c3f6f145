"""GPU parity of the generalized impulse responses (ccmm_girf.hip; generateGIRF2linear.m /
generateGIRF2blockhybrid.m:199-259 with antitheticSim and simVAR*) against the oracle
(oracle/ccmm_oracle_girf.girf_draw) on common random numbers, and the linear model's exact
property at the reference size: the antithetic mean of a linear simulation is the
deterministic path, so +shock minus baseline is the impulse response invA e1 shock11
propagated by the companion matrix."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gi():
    from oracle import ccmm_oracle_girf
    return ccmm_oracle_girf


def _draws(rng, N, p, M, bh, Ny):
    """M random stable draws: PAI K x N x M, invA (unit lower), sqrtPHI, SV0, Xjumpoff."""
    K = 1 + N * p
    PAI = np.zeros((K, N, M))
    invA = np.zeros((N, N, M))
    sqrtPHI = np.zeros((N, N, M))
    for m in range(M):
        PAI[0, :, m] = 0.1 * rng.standard_normal(N)
        for l in range(p):
            PAI[1 + l * N:1 + (l + 1) * N, :, m] = (0.5 / (l + 1) ** 2) * np.eye(N) + \
                0.03 * rng.standard_normal((N, N))
        invA[..., m] = np.eye(N) + np.tril(0.2 * rng.standard_normal((N, N)), -1)
        sqrtPHI[..., m] = np.tril(0.02 * rng.standard_normal((N, N)), -1) + np.diag(0.05 + 0.1 * rng.random(N))
    SV0 = 0.5 + rng.random((N, M))
    ns = K + (Ny * p if bh else 0)
    Xj = np.zeros((ns, M))
    Xj[0] = 1.0
    Xj[1:] = 0.3 * rng.standard_normal((ns - 1, M)) + 0.2
    return PAI, invA, sqrtPHI, SV0, Xj


@pytest.mark.parametrize("bh", [False, True])
def test_girf_crn_toy(ctx, gi, bh):
    rng = np.random.default_rng(7 + bh)
    N, p, H, nsim, M = 5, 2, 9, 6, 3
    yields = np.array([False, False, True, True, True])
    actual = ~yields
    cum = np.array([True, False, False, False, True])
    PAI, invA, sqrtPHI, SV0, Xj = _draws(rng, N, p, M, bh, int(yields.sum()))
    z = rng.standard_normal((N, H, nsim, M))
    svz = rng.standard_normal((N, H, nsim, M))
    got = ctx.girf(PAI, invA, sqrtPHI, SV0, Xj, H, nsim, 0.7, bh=bh, actual=actual, ndxYields=yields,
                   elb=0.25, cumcode=cum, np_=12, z=z, svz=svz)
    for m in range(M):
        want = gi.girf_draw(PAI[..., m], invA[..., m], sqrtPHI[..., m], SV0[:, m], Xj[:, m], z[..., m],
                            svz[..., m], 0.7, cum, 12, bh=bh, actual=actual, yields=yields, elb=0.25)
        for sc in range(3):
            err = np.max(np.abs(got[:, :, sc, m] - want[sc]) / np.maximum(np.abs(want[sc]), 1.0))
            assert err < 1e-12, (m, sc, err)


def test_girf_linear_reference_size(ctx, gi):
    """N = 20, p = 12, H = 120, 1000 shock paths, 8 draws, Philox: +shock - baseline and
    baseline - (-shock) equal the deterministic impulse response (antithetic cancellation)."""
    rng = np.random.default_rng(3)
    N, p, H, nsim, M = 20, 12, 120, 1000, 8
    PAI, invA, sqrtPHI, SV0, Xj = _draws(rng, N, p, M, False, 0)
    cum = np.zeros(N, bool)
    cum[:4] = True
    out = ctx.girf(PAI, invA, sqrtPHI, SV0, Xj, H, nsim, 1.0, cumcode=cum, np_=12, seed=11)
    assert np.all(np.isfinite(out))
    for m in range(M):
        A = gi.companion(PAI[..., m], N, p)
        x = np.zeros(A.shape[0])
        x[1:1 + N] = invA[:, 0, m]
        irf = np.zeros((N, H))
        for h in range(H):
            irf[:, h] = x[1:1 + N]
            x = A @ x
        irf[cum] = np.cumsum(irf[cum], axis=1) / 12
        scale = max(np.max(np.abs(out[:, :, 0, m])), 1.0)
        assert np.max(np.abs(out[:, :, 1, m] - out[:, :, 0, m] - irf)) < 1e-10 * scale
        assert np.max(np.abs(out[:, :, 0, m] - out[:, :, 2, m] - irf)) < 1e-10 * scale


def test_generate_girf_driver_linear(pkg, gi, fred):
    """samplers.generateGIRF (generateGIRF2linear.m:176-283) on synthetic kept draws: the
    median IRF over the draws equals the median of the deterministic responses."""
    rng = np.random.default_rng(5)
    N, p, M, H = 20, 12, 16, 24
    PAI, invA, sqrtPHI, SV0, _ = _draws(rng, N, p, M, False, 0)
    PHI = np.einsum("ijm,kjm->ikm", sqrtPHI, sqrtPHI)
    vech = np.array([[PHI[i, j, m] for j in range(N) for i in range(N) if i >= j] for m in range(M)])
    T = len(fred["ydates"]) - p
    sqrtht = np.repeat(SV0.T[:, None, :], T, axis=1)
    irfDate = fred["ydates"][-30]
    res = pkg.samplers.generateGIRF(fred["data"], fred["ydates"], irfDate, np.moveaxis(PAI, -1, 0),
                                    np.moveaxis(invA, -1, 0), vech, sqrtht, p=p, shock11=0.5,
                                    irfNdraws=64, irfHorizon=H, cumcode=fred["cumcode"])
    irfs = np.zeros((N, H, M))
    for m in range(M):
        A = gi.companion(PAI[..., m], N, p)
        x = np.zeros(A.shape[0])
        x[1:1 + N] = 0.5 * invA[:, 0, m]
        for h in range(H):
            irfs[:, h, m] = x[1:1 + N]
            x = A @ x
        irfs[fred["cumcode"], :, m] = np.cumsum(irfs[fred["cumcode"], :, m], axis=1) / 12
    want = np.median(irfs, axis=2)
    assert np.max(np.abs(res["IRF1plus"] - want)) < 1e-9 * max(1.0, np.abs(want).max())
    assert np.max(np.abs(res["IRF1minus"] + want)) < 1e-9 * max(1.0, np.abs(want).max())
    assert res["IRF1plusTails"].shape == (N, H, 2)


@pytest.mark.parametrize("bh", [False, True])
def test_girf_reference_shape_crn(ctx, gi, bh):
    """N = 20, p = 12 (the specialised aligned-layout kernel k_girf_fast) against the oracle
    on common random numbers: 2 draws x 5 shock paths x 30 horizons."""
    rng = np.random.default_rng(21 + bh)
    N, p, H, nsim, M = 20, 12, 30, 5, 2
    yields = np.zeros(N, bool)
    yields[[14, 15, 16, 17, 18, 19]] = True
    PAI, invA, sqrtPHI, SV0, Xj = _draws(rng, N, p, M, bh, 6)
    z = rng.standard_normal((N, H, nsim, M))
    svz = rng.standard_normal((N, H, nsim, M))
    cum = np.zeros(N, bool)
    cum[:5] = True
    got = ctx.girf(PAI, invA, sqrtPHI, SV0, Xj, H, nsim, 0.11, bh=bh, actual=~yields, ndxYields=yields,
                   elb=0.25, cumcode=cum, np_=12, z=z, svz=svz)
    for m in range(M):
        want = gi.girf_draw(PAI[..., m], invA[..., m], sqrtPHI[..., m], SV0[:, m], Xj[:, m], z[..., m],
                            svz[..., m], 0.11, cum, 12, bh=bh, actual=~yields, yields=yields, elb=0.25)
        for sc in range(3):
            err = np.max(np.abs(got[:, :, sc, m] - want[sc]) / np.maximum(np.abs(want[sc]), 1.0))
            assert err < 1e-12, (m, sc, err)


def _hybrid_draws(rng, N, p, M, Ns):
    """Hybrid PAI (K + Ns p) x N x M: the linear draws plus small coefficients on the Ns p
    actual-rate lags (Xffrlags, mcmcVARhybridGibbs.m:74-84)."""
    PAI, invA, sqrtPHI, SV0, _ = _draws(rng, N, p, M, False, 0)
    K = 1 + N * p
    PAIh = np.concatenate([PAI, 0.05 * rng.standard_normal((Ns * p, N, M))], axis=0)
    Xj = np.zeros((K + Ns * p, M))
    Xj[0] = 1.0
    Xj[1:] = 0.3 * rng.standard_normal((K + Ns * p - 1, M)) + 0.2
    return PAIh, invA, sqrtPHI, SV0, Xj


@pytest.mark.parametrize("N,p,yidx,sidx", [(5, 2, [2, 3, 4], [2, 3]),
                                            (20, 12, [14, 15, 16, 17, 18, 19], [14, 15, 16])])
def test_girf_hybrid_crn(ctx, gi, N, p, yidx, sidx):
    """generateGIRF2hybrid.m (simVARhybrid, :361-386) against the oracle on common random numbers:
    the state carries the Ns shadow-rate variables' actual-rate lags, the companion rows are the
    full hybrid PAI, the output floors every yield.  N = 20, p = 12, Ns = 3 runs the specialised
    kernel (ring padded to 4 rows), the toy shape the table-driven one."""
    rng = np.random.default_rng(40 + N)
    H, nsim, M = 14, 5, 2
    yields = np.zeros(N, bool)
    yields[yidx] = True
    shadow = np.zeros(N, bool)
    shadow[sidx] = True
    PAI, invA, sqrtPHI, SV0, Xj = _hybrid_draws(rng, N, p, M, int(shadow.sum()))
    z = rng.standard_normal((N, H, nsim, M))
    svz = rng.standard_normal((N, H, nsim, M))
    cum = np.zeros(N, bool)
    cum[0] = True
    got = ctx.girf(PAI, invA, sqrtPHI, SV0, Xj, H, nsim, 0.3, hybrid=True, ndxShadow=shadow, ndxYields=yields,
                   elb=0.25, cumcode=cum, np_=12, z=z, svz=svz, p=p)
    for m in range(M):
        want = gi.girf_draw(PAI[..., m], invA[..., m], sqrtPHI[..., m], SV0[:, m], Xj[:, m], z[..., m],
                            svz[..., m], 0.3, cum, 12, yields=yields, elb=0.25, shadow=shadow, p=p)
        for sc in range(3):
            err = np.max(np.abs(got[:, :, sc, m] - want[sc]) / np.maximum(np.abs(want[sc]), 1.0))
            assert err < 1e-12, (m, sc, err)
