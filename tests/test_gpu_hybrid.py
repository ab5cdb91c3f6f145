"""GPU parity of the hybrid shadow-rate sweep (mcmcVARhybridGibbs.m:362-539) against
oracle/ccmm_oracle_hybrid.hybrid_sweep: CTA on the chain's K = 1 + N p + Ns p design,
A, SV, PHI, the ELB Gibbs step with companion PAI(1:Kshadow,:) and Yhatactual =
Xffrlags PAIactual, and the X/Y rebuild; common random numbers per chain.  Parity
metric |Δ| / max(|x|, scale); the ELB comparison follows
test_gpu_bh.py (stable residual form, as-written distance reported)."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import hybrid_crn_flat, random_state, toy_hybrid_setup

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hy():
    from oracle import ccmm_oracle_hybrid
    return ccmm_oracle_hybrid


def _real_hs(hy, oracle, fred):
    ndxS, _, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    return hy.hybrid_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, mpm,
                           0.25, e0)


def _chains(pkg, ctx, hs, B, crn, cap):
    lin = hs.lin
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=crn, model=pkg.MODEL_HYBRID,
                    Ns=len(hs.ndxS), elbTmax=hs.elbT, elb_gibbsburn=hs.gibbsburn, elb=hs.ELB,
                    store_capacity=cap)
    assert ch.cfg.K == lin.K
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(hs.ndxS, None)
    ch.set_elb_slot(0, hs.elbT0, hs.sNaN)
    return ch


def _run_check(pkg, ctx, oracle, hy, hs, B, nsweeps, seed, tol_pai, tol_s, cta_form="mirror"):
    lin = hs.lin
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=seed + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(seed)
    crns = [[hy.hybrid_draw_crn(rng, hs) for _ in range(nsweeps)] for _ in range(B)]
    ch = _chains(pkg, ctx, hs, B, True, nsweeps)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    flat = np.stack([np.stack([hybrid_crn_flat(hy, crns[c][m], hs) for m in range(nsweeps)], -1)
                     for c in range(B)], -1)
    assert flat.shape[0] == ch.crn_len
    ch.sweep(nsweeps, crn=flat, store=True)
    got = ch.get_state()
    S = ch.get_shadowrate()
    X, Y = ch.get_xy()
    draws = ch.get_draws()
    for c in range(B):
        st = sts[c]
        for m in range(nsweeps):
            prev = st
            st = hy.hybrid_sweep(st, hs, crns[c][m], elb_impl="both", cta_form=cta_form)
            np.testing.assert_allclose(draws["PAI_all"][m, :, :, c], st["PAI"], rtol=0,
                                       atol=max(tol_pai, 1e-12) * max(1.0, np.abs(st["PAI"]).max()))
        _, _, sd = oracle.cta(prev["Y"], prev["X"], lin.N, lin.K, prev["A"], prev["sqrtht"],
                              lin.iVdiag, lin.iVb, prev["PAI"], np.zeros((lin.K, lin.N)),
                              return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], prev["sqrtht"])),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3),
             "shadowrate": rel_err(S[:, :, c], st["shadowrate"], 0.1),
             "Y": rel_err(Y[..., c], st["Y"], 0.1),
             "X": rel_err(X[..., c], st["X"], 0.1)}
        qr_gap = float(np.max(np.abs(st["shadowrate_qr"] - st["shadowrate"])))
        gpu_qr = float(np.max(np.abs(S[:, :, c] - st["shadowrate_qr"])))
        print("chain", c, e, "as-written gap: oracle", qr_gap, "gpu", gpu_qr, "| PAI entries differing",
              int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        assert gpu_qr <= qr_gap + 1e-6
        assert e["shadowrate"] < tol_s and e["X"] < tol_s and e["Y"] < tol_s, e
        assert max(e["PAI"], e["A"], e["sqrtht"], e["sqrtPHI"]) < tol_pai, e
        assert np.all(S[:, :, c][hs.sNaN] <= hs.ELB + 1e-12)
        np.testing.assert_array_equal(X[:, hs.Kshadow:, c], hs.Xffrlags)  # fixed actual-rate lags


def test_hybrid_sweep_crn_toy(pkg, ctx, oracle, hy):
    """N=5, p=2, two shadow rates (K = 15): 3 chains x 2 chained sweeps against the oracle with CTA in
    the device's large-system operation order (oracle/cta_big_mirror.c)."""
    hs = toy_hybrid_setup(hy)
    _run_check(pkg, ctx, oracle, hy, hs, B=3, nsweeps=2, seed=70, tol_pai=1e-9, tol_s=1e-9)


def test_hybrid_sweep_crn_real(pkg, ctx, oracle, hy, fred):
    """Real data, ELB 0.25, p = 12: K = 277 (KP = 320, the large-system kernels k_gram_big / k_chol_big
    / k_cta_solve_big), elbT = 165, three shadow rates; one sweep from a smooth-volatility state against
    the oracle with CTA in the device's operation order: the north star's 1e-9."""
    hs = _real_hs(hy, oracle, fred)
    _run_check(pkg, ctx, oracle, hy, hs, B=2, nsweeps=1, seed=80, tol_pai=1e-9, tol_s=1e-9)


def test_hybrid_sweep_crn_real_as_written(pkg, ctx, oracle, hy, fred):
    """The same sweep against CTA.m as written (kron-materialised X_j, explicit inverse): the
    summation orders differ, ~1e-8 posterior sd at this conditioning."""
    hs = _real_hs(hy, oracle, fred)
    _run_check(pkg, ctx, oracle, hy, hs, B=2, nsweeps=1, seed=80, tol_pai=1e-7, tol_s=1e-6, cta_form="kron")


def test_hybrid_philox_batch(pkg, ctx, oracle, hy, fred):
    """Production mode (Philox): 8 chains from the reference initialisation (:351-359);
    censored cells at or below the ELB, uncensored cells equal the data."""
    hs = _real_hs(hy, oracle, fred)
    lin = hs.lin
    B = 8
    ch = _chains(pkg, ctx, hs, B, False, 2)
    st = oracle.init_state(lin)
    ch.set_state(*[np.repeat(st[k][..., None], B, -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    ch.sweep(2, store=False)
    ch.sweep(2, store=True)
    d = ch.get_draws()
    sr = d["shadowrate_all"]
    assert sr.shape == (2, 3, hs.elbT, B) and np.all(np.isfinite(sr))
    cens = np.broadcast_to(hs.sNaN[None, :, :, None], sr.shape)
    assert np.all(sr[cens] <= 0.25 + 1e-12)
    Yw = np.broadcast_to(lin.Y[hs.elbT0:, hs.ndxS].T[None, :, :, None], sr.shape)
    np.testing.assert_array_equal(sr[~cens], Yw[~cens])
    assert d["PAI_all"].shape == (2, lin.K, lin.N, B) and np.all(np.isfinite(d["PAI_all"]))


def test_lag_twin_bit_identical(pkg, ctx, oracle, hy, fred):
    """The large path's Gram and solve on the column-major lag twin of X (option big_lagx = 1, the
    default) against X itself (0): the same products in the same order, so the same draws bit for bit
    -- over three sweeps, so the ELB step's rebuild of the twin (k_elb_rebuild) is exercised."""
    hs = _real_hs(hy, oracle, fred)
    lin = hs.lin
    out = {}
    for lx in (1, 0):
        ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=4, crn=False, seed=11, model=pkg.MODEL_HYBRID,
                        Ns=len(hs.ndxS), elbTmax=hs.elbT, elb_gibbsburn=hs.gibbsburn, elb=hs.ELB,
                        store_capacity=3, options={"big_lagx": lx})
        ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
        ch.set_elb_model(hs.ndxS, None)
        ch.set_elb_slot(0, hs.elbT0, hs.sNaN)
        sts = [random_state(oracle, lin, seed=40 + c) for c in range(4)]
        ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
        ch.sweep(3, store=True)
        out[lx] = (ch.get_state(), ch.get_shadowrate(), ch.get_status())
    assert np.all(out[1][2] & ~1 == 0) and np.all(out[0][2] & ~1 == 0)
    for k in out[1][0]:
        np.testing.assert_array_equal(out[1][0][k], out[0][0][k], err_msg=k)
    np.testing.assert_array_equal(out[1][1], out[0][1])
