"""ccmm_gibbs_shadowrates with a general impact matrix (gibbsdrawShadowrates.m:49-58, 74-95: the reference
QR-factors M = Cpowerp Psi diag(SVol) for any Psi; every in-tree caller passes invA, lower triangular).
A dense Psi(2:Ny+1, :) is inverted on the host by Gauss-Jordan with partial pivoting and the device ELB
conditionals run on the full structural matrix A = Psi(2:Ny+1, :)^-1.  Toy VAR (Ny = 4, p = 2, Ns = 2,
T = 40, a censored stretch with a gap), 100 burn-in passes + 1 draw, common uniforms, against the oracle's
restatement as written (QR smoothing weights, oracle.gibbsdraw_shadowrates): drawTruncNormal branch flags
bit-exact, draws within 1e-9 (the toy companion is stable, so the as-written form is accurate)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(seed, dense, T=40):
    rng = np.random.default_rng(seed)
    Ny, p, Ns = 4, 2, 2
    K = Ny * p + 1
    PAI = np.zeros((K, Ny))
    PAI[0] = rng.uniform(-0.2, 0.2, Ny)
    for l in range(p):
        PAI[1 + l * Ny:1 + (l + 1) * Ny] = (0.5 / (l + 1)) * np.eye(Ny) + 0.05 * rng.standard_normal((Ny, Ny))
    C = np.zeros((K, K))
    C[0, 0] = 1.0
    C[1:1 + Ny, :] = PAI.T
    C[1 + Ny:, 1:1 + Ny * (p - 1)] = np.eye(Ny * (p - 1))
    Psi = np.zeros((K, Ny))
    Psi[1:1 + Ny] = np.eye(Ny) + np.tril(0.3 * rng.standard_normal((Ny, Ny)), -1)
    if dense:
        Psi[1:1 + Ny] += np.triu(0.3 * rng.standard_normal((Ny, Ny)), 1)
    ndxS = np.zeros(Ny, bool)
    ndxS[:Ns] = True
    sNaN = np.zeros((Ns, T), bool)
    sNaN[:, 8:30] = True
    sNaN[1, 12:15] = False
    Y = rng.normal(size=(Ny, T)) + 1.0
    Y[:Ns][sNaN] = 0.2
    STATE0 = np.concatenate([[1.0], 1.0 + rng.normal(size=Ny * p)])
    YHAT0 = 0.1 * rng.normal(size=(Ny, T))
    SVol = np.exp(0.2 * rng.normal(size=(Ny, T)))
    u = rng.random((Ns, T, 101))
    return Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, u


@pytest.mark.parametrize("dense", [True, False])
def test_gibbs_shadowrates_general_psi(ctx, oracle, dense):
    B = 2
    cases = [_case(30 + c, dense) for c in range(B)]
    stk = [np.stack([cs[k] for cs in cases], -1) for k in (0, 1, 2, 6, 7, 8, 9)]
    Y, STATE0, YHAT0, C, Psi, SVol, u = stk
    ndxS, sNaN, p = cases[0][3], cases[0][4], cases[0][5]
    got, fl = ctx.gibbs_shadowrates(Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, 0.25, burnin=100, u=u,
                                    flags=True)
    for c in range(B):
        Yc, S0, YH, _, _, _, Cc, Pc, SV, uc = cases[c]
        assert dense == bool(np.any(np.triu(Pc[1:5], 1)))
        want, wfl = oracle.gibbsdraw_shadowrates(Yc, S0, YH, ndxS, sNaN, p, Cc, Pc, SV, 0.25, 1, 100, uc,
                                                 return_flags=True)
        np.testing.assert_array_equal(fl[..., c], wfl)
        err = np.max(np.abs(got[:, :, 0, c][sNaN] - want[:, :, 0][sNaN]) / np.maximum(np.abs(want[:, :, 0][sNaN]), 0.1))
        print(f"dense {dense} chain {c}: max rel |draw - oracle| {err:.2e}, {int(np.count_nonzero(wfl))} flags")
        assert err < 1e-9
        assert np.all(got[:, :, 0, c][sNaN] <= 0.25)


def test_gibbs_shadowrates_singular_psi_is_an_error(ctx):
    Y, STATE0, YHAT0, ndxS, sNaN, p, C, Psi, SVol, u = _case(40, True)
    Psi[2, :] = Psi[1, :]  # two equal rows of Psi(2:Ny+1, :)
    with pytest.raises(RuntimeError, match="singular"):
        ctx.gibbs_shadowrates(Y[..., None], STATE0[:, None], YHAT0[..., None], ndxS, sNaN, p, C[..., None],
                              Psi[..., None], SVol[..., None], 0.25, burnin=2, u=u[:, :, :3, None])
