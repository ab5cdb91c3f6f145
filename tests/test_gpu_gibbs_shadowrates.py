"""C-ABI drop-in of gibbsdrawShadowrates (ccmm_gibbs_shadowrates, gibbsdrawShadowrates.m:1-245)
on the real C3 window (fredblockMD20, ELB 0.25, p = 12: elbT = 165 months, three shadow
rates, 109 censored months), 100 + 1 passes with common uniforms, three independent calls
batched.  Compared with oracle.gibbsdraw_shadowrates (the QR formulation as written) and
with its stable residual form (oracle/elb_fast.py, the form the device evaluates): draws in
units of max(|x|, 0.1), drawTruncNormal branch flags bit-exact."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _c3(oracle, fred):
    from oracle import ccmm_oracle_bh as bh
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    return bh, bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO,
                           mpm, 0.25, e0)


@pytest.mark.parametrize("burn,tol", [(0, 1e-7), (100, 1e-6)])
def test_gibbs_shadowrates_c3(ctx, oracle, fred, burn, tol):
    """The C3 states here have a shadow companion spectral radius ~1.01: the deterministic
    path Y0 grows to ~250 over the window and the as-written Ytilde = Y - Y0 cancels, so the
    oracle's own two forms (QR as written, stable residual form) differ by ~3.5e-7.  Bars:
    GPU vs the stable form 1e-7 (one pass) / 1e-6 (101 passes, each conditioning on the
    previous one's draws, as the in-sweep ELB step of tests/test_gpu_bh.py); GPU vs the
    as-written form no further than the oracle's own gap; branch flags bit-exact."""
    from oracle import elb_fast as F
    bh, bs = _c3(oracle, fred)
    lin = bs.lin
    st = bh.bh_init_state(bs)
    B = 3
    ins = []
    for c in range(B):
        rng = np.random.default_rng(70 + c)
        A = np.eye(lin.N) + np.tril(rng.uniform(-0.2, 0.2, (lin.N, lin.N)), -1)
        sqrtht = st["sqrtht"] * np.exp(np.cumsum(0.02 * rng.standard_normal((lin.T, lin.N)), axis=0))
        C, Psi, SVol, Yhat = bh.elb_state_space(bs, st["PAI"], np.linalg.inv(A), sqrtht)
        Y = st["Y"][bs.elbT0:, :].T.copy()
        u = rng.random((len(bs.ndxS), bs.elbT, burn + 1))
        ins.append((Y, bs.X0, Yhat, C, Psi, SVol, u))
    stk = [np.stack([x[k] for x in ins], -1) for k in range(7)]
    got, fl = ctx.gibbs_shadowrates(stk[0], stk[1], stk[2], bs.ndxSmask, bs.sNaN, lin.p, stk[3],
                                    stk[4], stk[5], 0.25, burnin=burn, u=stk[6], flags=True)
    assert got.shape == (len(bs.ndxS), bs.elbT, 1, B)
    for c in range(B):
        Y, X0, Yhat, C, Psi, SVol, u = ins[c]
        want, wfl = oracle.gibbsdraw_shadowrates(Y, X0, Yhat, bs.ndxSmask, bs.sNaN, lin.p, C, Psi,
                                                 SVol, 0.25, 1, burn, u, return_flags=True)
        stab = F.gibbsdraw_shadowrates_stable(Y, X0, Yhat, bs.ndxSmask, bs.sNaN, lin.p, C, Psi,
                                              SVol, 0.25, 1, burn, u)
        e_qr = rel_err(got[:, :, 0, c], want[:, :, 0], 0.1)
        e_st = rel_err(got[:, :, 0, c], stab[:, :, 0], 0.1)
        gap = rel_err(stab[:, :, 0], want[:, :, 0], 0.1)
        print("chain", c, "vs as-written", e_qr, "vs stable", e_st, "oracle gap", gap)
        assert e_st < tol and e_qr <= gap + tol
        np.testing.assert_array_equal(fl[..., c], wfl)
        assert np.all(got[:, :, 0, c][bs.sNaN] <= 0.25 + 1e-12)


def test_gibbs_shadowrates_dimension_mismatch(ctx, oracle, fred):
    """sum(ndxS) != rows of sNaN: gibbsdrawShadowrates.m:50-52 'dimension mismatch'."""
    bh, bs = _c3(oracle, fred)
    lin = bs.lin
    st = bh.bh_init_state(bs)
    C, Psi, SVol, Yhat = bh.elb_state_space(bs, st["PAI"], np.eye(lin.N), st["sqrtht"])
    with pytest.raises(RuntimeError, match="rc=-1"):
        ctx.gibbs_shadowrates(st["Y"][bs.elbT0:, :].T, bs.X0, Yhat, bs.ndxSmask, bs.sNaN[:2], lin.p,
                              C, Psi, SVol, 0.25, burnin=2)


@pytest.mark.parametrize("burn", [0, 100])
def test_gibbs_shadowrates_c3_drawn_state(ctx, oracle, fred, burn):
    """The same drop-in on states the sampler visits: PAI, invA and sqrtht after one block-hybrid
    sweep from a smooth-volatility state, instead of the OLS coefficients of the reference
    initialisation above.  The GPU agrees with the oracle's stable form to the north star's 1e-9
    over 1 and 101 passes (measured 3e-14); branch flags bit-exact."""
    from oracle import elb_fast as F
    from helpers import random_state
    bh, bs = _c3(oracle, fred)
    lin = bs.lin
    B = 2
    ins, rho = [], []
    for c in range(B):
        rng = np.random.default_rng(90 + c)
        st = random_state(oracle, lin, seed=90 + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        st = bh.bh_sweep(st, bs, bh.bh_draw_crn(rng, bs), elb_impl="stable")
        C, Psi, SVol, Yhat = bh.elb_state_space(bs, st["PAI"], st["invA"], st["sqrtht"])
        rho.append(float(np.max(np.abs(np.linalg.eigvals(C)))))
        Y = st["Y"][bs.elbT0:, :].T.copy()
        u = rng.random((len(bs.ndxS), bs.elbT, burn + 1))
        ins.append((Y, bs.X0, Yhat, C, Psi, SVol, u))
    stk = [np.stack([x[k] for x in ins], -1) for k in range(7)]
    got, fl = ctx.gibbs_shadowrates(stk[0], stk[1], stk[2], bs.ndxSmask, bs.sNaN, lin.p, stk[3],
                                    stk[4], stk[5], 0.25, burnin=burn, u=stk[6], flags=True)
    for c in range(B):
        Y, X0, Yhat, C, Psi, SVol, u = ins[c]
        stab, sfl = F.gibbsdraw_shadowrates_stable(Y, X0, Yhat, bs.ndxSmask, bs.sNaN, lin.p, C, Psi, SVol, 0.25,
                                                   1, burn, u, return_flags=True)
        e_st = rel_err(got[:, :, 0, c], stab[:, :, 0], 0.1)
        print("chain", c, "companion spectral radius", rho[c], "vs stable", e_st)
        assert e_st < 1e-9
        np.testing.assert_array_equal(fl[..., c], sfl)
