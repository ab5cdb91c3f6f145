"""GPU parity of the block-hybrid shadow-rate sweep (mcmcVARshadowrateBlockHybrid.m:322-523)
against oracle/ccmm_oracle_bh.bh_sweep (CTAsys, A, SV, PHI, the ELB Gibbs step with
100 + 1 passes, X/Y rebuild), common random numbers per chain.  Parity metric:
|Δ| / max(|x|, scale).

The ELB step is compared with the oracle's stable residual form
(elb_fast.gibbsdraw_shadowrates_stable, equal to gibbsdrawShadowrates in exact
arithmetic and to its QR evaluation at 1e-10 when Y0 stays bounded, see
tests/test_oracle_bh.py).  When a chain's shadow companion matrix is explosive
the as-written QR evaluation itself is off by O(0.1) late in the window; the
distance GPU <-> as-written is then reported and must not exceed the oracle's
own stable <-> as-written distance."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import bh_crn_flat, random_state, toy_bh_setup

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bh():
    from oracle import ccmm_oracle_bh
    return ccmm_oracle_bh


def _real_bs(bh, oracle, fred):
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    return bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                       0.25, e0)


def _run(pkg, ctx, oracle, bh, bs, B, nsweeps, seed, cta_form="mirror", shadowrate_model=False):
    lin = bs.lin
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=seed + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(seed)
    crns = [[bh.bh_draw_crn(rng, bs) for _ in range(nsweeps)] for _ in range(B)]
    model = pkg.MODEL_SHADOWRATE if shadowrate_model else pkg.MODEL_BLOCKHYBRID
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=True, model=model,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                    store_capacity=nsweeps)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, None if shadowrate_model else bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([bh_crn_flat(bh, crns[c][m], bs) for m in range(nsweeps)], -1)
                     for c in range(B)], -1)
    ch.record_elb_flags(True)
    ch.sweep(nsweeps, crn=flat, store=True)
    got = ch.get_state()
    got["kai"] = ch.get_kai()
    got["elb_flags"] = ch.get_elb_flags()
    S = ch.get_shadowrate()
    X, Y = ch.get_xy()
    draws = ch.get_draws()
    want = []
    for c in range(B):
        st = sts[c]
        hist = []
        for m in range(nsweeps):
            prev_sqrtht = st["sqrtht"]
            st = bh.bh_sweep(st, bs, crns[c][m], elb_impl="both", return_flags=True, cta_form=cta_form)
            hist.append(st["shadowrate"])
        st["prev_sqrtht"] = prev_sqrtht
        want.append((st, hist))
    return got, S, X, Y, draws, want


def _check(oracle, bs, got, S, X, Y, draws, want, tol_pai, tol_s):
    lin = bs.lin
    for c, (st, hist) in enumerate(want):
        XX = np.empty((lin.T, lin.K, lin.N))
        XX[:, :, bs.actualrateBlock] = bs.Xactual[:, :, None]
        XX[:, :, ~bs.actualrateBlock] = st["X"][:, :, None]
        _, _, sd = oracle.cta_sys(st["Y"], XX, lin.N, lin.K, lin.T, st["A"], st["sqrtht"],
                                  lin.iVdiag, lin.iVb, st["PAI"], np.zeros((lin.K, lin.N)),
                                  return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"],
                          oracle.a_step_sd(st["RESID"], st["prev_sqrtht"])),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3),
             "shadowrate": rel_err(S[:, :, c], st["shadowrate"], 0.1),
             "Y": rel_err(Y[..., c], st["Y"], 0.1),
             "X": rel_err(X[..., c], st["X"], 0.1)}
        qr_gap = float(np.max(np.abs(st["shadowrate_qr"] - st["shadowrate"])))
        gpu_qr = float(np.max(np.abs(S[:, :, c] - st["shadowrate_qr"])))
        print("chain", c, e, "as-written gap: oracle", qr_gap, "gpu", gpu_qr,
              "| PAI entries differing", int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        assert gpu_qr <= qr_gap + 1e-6
        assert e["shadowrate"] < tol_s and e["X"] < tol_s and e["Y"] < tol_s, e
        assert max(e["PAI"], e["A"], e["sqrtht"], e["sqrtPHI"]) < tol_pai, e
        sN = bs.sNaN
        assert np.all(S[:, :, c][sN] <= bs.ELB + 1e-12)
        # KSC indicators and drawTruncNormal branches of the last sweep: bit-exact (the
        # branches against the stable form the device evaluates; against the as-written QR
        # form too where that form is itself accurate)
        np.testing.assert_array_equal(got["kai"][..., c], st["kai"])
        np.testing.assert_array_equal(got["elb_flags"][:, :bs.elbT, :, c], st["elb_flags_stable"])
        if qr_gap < 1e-9:
            np.testing.assert_array_equal(got["elb_flags"][:, :bs.elbT, :, c], st["elb_flags"])
        for m, sr in enumerate(hist):  # stored draws (shadowrate_all, :542)
            assert rel_err(draws["shadowrate_all"][m, :, :, c], sr, 0.1) < max(tol_s, 1e-6)


def test_bh_sweep_crn_toy(pkg, ctx, oracle, bh):
    """N=5, p=2, two shadow rates (one with gaps in its censoring), one other yield; two chained
    sweeps against the oracle with CTAsys in the device's operation order (cta_form="mirror")."""
    bs = toy_bh_setup(bh)
    out = _run(pkg, ctx, oracle, bh, bs, B=3, nsweeps=2, seed=40)
    _check(oracle, bs, *out, tol_pai=1e-9, tol_s=1e-9)


def test_bh_sweep_crn_real(pkg, ctx, oracle, bh, fred):
    """Config C3 data (fredblockMD20, ELB 0.25, p = 12): elbT = 165, 109 censored months, three
    shadow rates; one sweep from a smooth-volatility state, the oracle's CTAsys in the device's
    operation order (oracle/cta_mirror.cta with the actual-rate and shadow-rate designs): the north
    star's 1e-9 (measured: PAI bit-exact, the rest <= 6e-13), drawTruncNormal branches bit-exact."""
    bs = _real_bs(bh, oracle, fred)
    out = _run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=1, seed=60)
    _check(oracle, bs, *out, tol_pai=1e-9, tol_s=1e-9)


def test_bh_sweep_crn_real_two_sweeps(pkg, ctx, oracle, bh, fred):
    """As test_bh_sweep_crn_real over two chained sweeps: the second sweep's CTAsys conditions on
    A / sqrtht / shadow rates that differ from the oracle's by rounding (~1e-13), which the
    real-data conditioning (cond(iV_post) ~ 1e9..1e13) amplifies; the bar stays 1e-9."""
    bs = _real_bs(bh, oracle, fred)
    out = _run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=2, seed=61)
    _check(oracle, bs, *out, tol_pai=1e-9, tol_s=1e-9)


def test_bh_sweep_crn_real_as_written(pkg, ctx, oracle, bh, fred):
    """The same sweep against CTAsys.m as written (kron-materialised X_j, explicit inverse): only
    the summation orders differ, which at this conditioning moves the draws by ~1e-8 posterior sd
    (SURVEY §7)."""
    bs = _real_bs(bh, oracle, fred)
    out = _run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=1, seed=60, cta_form="kron")
    _check(oracle, bs, *out, tol_pai=1e-7, tol_s=1e-6)


def test_bh_philox_batch(pkg, ctx, oracle, bh, fred):
    """Production mode on C3 data: 16 chains, Philox, stored draws; censored cells
    stay at or below the ELB, uncensored cells equal the data, chains differ."""
    bs = _real_bs(bh, oracle, fred)
    lin = bs.lin
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"],
                            oracle.set_minnesota_mean(fred["ncode"]), True)
    B = 16
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb=0.25, store_capacity=3)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(3, store=False)
    ch.sweep(3, store=True)
    d = ch.get_draws()
    sr = d["shadowrate_all"]
    assert sr.shape == (3, 3, bs.elbT, B)
    assert np.all(np.isfinite(sr))
    cens = np.broadcast_to(bs.sNaN[None, :, :, None], sr.shape)
    assert np.all(sr[cens] <= 0.25 + 1e-12)
    Yw = np.broadcast_to(lin.Y[bs.elbT0:, bs.ndxS].T[None, :, :, None], sr.shape)
    np.testing.assert_array_equal(sr[~cens], Yw[~cens])
    assert np.std(sr[-1, 0, 30, :]) > 0
    for k in ("PAI_all", "PHI_all", "invA_all", "sqrtht_all"):
        assert np.all(np.isfinite(d[k]))


def test_bh_large_path_lag_twin_bit_identical(pkg, ctx, oracle, bh, fred):
    """CTAsys on the large path (option large_path = 1) with the Gram and solve reading the lag twins
    of the vintage's and the chain's X slabs (big_lagx = 1) against the designs themselves (0): the
    same draws bit for bit over three sweeps (the chain slabs' twins are rebuilt by the ELB step)."""
    bs = _real_bs(bh, oracle, fred)
    lin = bs.lin
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"],
                            oracle.set_minnesota_mean(fred["ncode"]), True)
    out = {}
    for lx in (1, 0):
        ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=4, crn=False, seed=9, model=pkg.MODEL_BLOCKHYBRID,
                        Ns=len(bs.ndxS), elbTmax=bs.elbT, elb=0.25, store_capacity=3,
                        options={"large_path": 1, "big_lagx": lx})
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
        ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
        st = pkg.model.initial_state(m, 4)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        ch.sweep(3, store=True)
        out[lx] = (ch.get_state(), ch.get_shadowrate(), ch.get_status())
    assert np.all(out[1][2] & ~1 == 0) and np.all(out[0][2] & ~1 == 0)
    for k in out[1][0]:
        np.testing.assert_array_equal(out[1][0][k], out[0][0][k], err_msg=k)
    np.testing.assert_array_equal(out[1][1], out[0][1])
