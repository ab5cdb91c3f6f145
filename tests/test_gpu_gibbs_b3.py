"""gibbsdrawShadowratesB3 on the device (ccmm_gibbs_shadowrates_b3) against the oracle's restatement
as written (oracle.gibbsdraw_shadowrates_b3: QR smoothing weights, gibbsdrawShadowratesB3.m:1-231,
itself pinned by tests/test_oracle_b3.py's likelihood KATs), common uniforms: a toy VAR (Ny = 4,
p = 2, Ns = 2) with a month-varying impact matrix B(:,:,t) and with a constant one, 100 burn-in
passes + 1 draw.  Every drawTruncNormal branch flag bit-exact, draws within 1e-9."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(seed, T=40, month_varying=True):
    rng = np.random.default_rng(seed)
    Ny, p, Ns = 4, 2, 2
    K = Ny * p + 1
    PAI = np.zeros((K, Ny))
    PAI[0] = rng.uniform(-0.2, 0.2, Ny)
    for l in range(p):
        PAI[1 + l * Ny:1 + (l + 1) * Ny] = (0.5 / (l + 1)) * np.eye(Ny) + 0.05 * rng.standard_normal((Ny, Ny))
    A = np.zeros((K, K))
    A[0, 0] = 1.0
    A[1:1 + Ny, :] = PAI.T
    A[1 + Ny:, 1:1 + Ny * (p - 1)] = np.eye(Ny * (p - 1))
    if month_varying:
        Bm = np.zeros((K, Ny, T))
        for t in range(T):
            Bm[1:1 + Ny, :, t] = np.eye(Ny) + np.tril(0.3 * rng.standard_normal((Ny, Ny)), -1)
    else:
        Bm = np.zeros((K, Ny))
        Bm[1:1 + Ny] = np.eye(Ny) + np.tril(0.3 * rng.standard_normal((Ny, Ny)), -1)
    ndxS = np.zeros(Ny, bool)
    ndxS[:Ns] = True
    sNaN = np.zeros((Ns, T), bool)
    sNaN[:, 8:30] = True
    sNaN[1, 12:15] = False
    Y = rng.normal(size=(Ny, T)) + 1.0
    Y[:Ns][sNaN] = 0.2
    STATE0 = np.concatenate([[1.0], 1.0 + rng.normal(size=Ny * p)])
    SVol = np.exp(0.2 * rng.normal(size=(Ny, T)))
    u = rng.random((Ns, T, 101))
    return Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, u


@pytest.mark.parametrize("month_varying", [True, False])
def test_b3_matches_oracle(pkg, ctx, oracle, month_varying):
    Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, u = _case(5, month_varying=month_varying)
    want, wfl = oracle.gibbsdraw_shadowrates_b3(Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, 0.25, 1, 100, u,
                                                return_flags=True)
    got, fl = ctx.gibbs_shadowrates_b3(Y[..., None], STATE0[:, None], ndxS, sNaN, p, A[..., None], Bm[..., None],
                                       SVol[..., None], 0.25, burnin=100, u=u[..., None], flags=True,
                                       month_varying=month_varying)
    np.testing.assert_array_equal(fl[..., 0][sNaN[:, :, None].repeat(101, 2)], wfl[sNaN[:, :, None].repeat(101, 2)])
    err = np.max(np.abs(got[:, :, 0, 0][sNaN] - want[:, :, 0][sNaN]))
    print(f"month-varying B {month_varying}: max |draw - oracle| {err:.2e}, "
          f"{int(np.count_nonzero(wfl))} flagged draws")
    assert err < 1e-9
    assert np.all(got[:, :, 0, 0][sNaN] <= 0.25)
    # the reference-signature mirror (samplers.gibbsdrawShadowratesB3) returns the same draws
    again = pkg.samplers.gibbsdrawShadowratesB3(Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, 0.25, 1, 100, u)
    np.testing.assert_array_equal(again, got[..., 0])


def test_b3_dense_B_matches_oracle(ctx, oracle):
    """A B(2:Ny+1, :) with an upper triangle (the function takes any impact matrix; its QR form factors
    M = Cpowerp B diag(SVol), gibbsdrawShadowratesB3.m:49-62): the device inverts it by Gauss-Jordan and
    runs the conditionals on the full structural matrix.  Flags bit-exact, draws within 1e-9."""
    Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, u = _case(6, month_varying=False)
    Bm[1:5, :] += np.triu(0.25 * np.random.default_rng(1).standard_normal((4, 4)), 1)
    want, wfl = oracle.gibbsdraw_shadowrates_b3(Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, 0.25, 1, 100, u,
                                                return_flags=True)
    got, fl = ctx.gibbs_shadowrates_b3(Y[..., None], STATE0[:, None], ndxS, sNaN, p, A[..., None], Bm[..., None],
                                       SVol[..., None], 0.25, burnin=100, u=u[..., None], flags=True)
    np.testing.assert_array_equal(fl[..., 0][sNaN[:, :, None].repeat(101, 2)], wfl[sNaN[:, :, None].repeat(101, 2)])
    err = np.max(np.abs(got[:, :, 0, 0][sNaN] - want[:, :, 0][sNaN]))
    print(f"dense B: max |draw - oracle| {err:.2e}")
    assert err < 1e-9
