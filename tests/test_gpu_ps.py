"""GPU parity of the acceptance-sampling branch of the ELB step
(mcmcVARshadowrateBlockHybrid.m:438-466; ccmm_ps.hip) against the oracle
(ccmm_oracle_bh.bh_sweep(use_ps=True): the precision sampler restated from the absent
VARTVPSVprecisionsamplerNaN, accept-first loop, Gibbs fallback), common random numbers
per chain.  The accepted proposal index (ndxAccept) must agree exactly; the draws within
the sweep tolerances of test_gpu_bh.py."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import random_state, synth_bh_data

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bh():
    from oracle import ccmm_oracle_bh
    return ccmm_oracle_bh


def _toy_bs(bh, window, seed=3, valley=False):
    """Toy block-hybrid panel; valley=True lets the shadow rates glide down to the ELB
    around the window (so the conditional means of the censored cells sit near it)."""
    N, p, Tobs, ndxS, ndxO = 5, 2, 150, (2, 3), (4,)
    data = synth_bh_data(N, p, Tobs, elb_window=window, ndxS=ndxS, seed=seed)
    if valley:
        a, b = window
        rng = np.random.default_rng(seed)
        for s in ndxS:
            lvl = np.full(Tobs, 0.9)
            lvl[a - 12:a] = np.linspace(0.9, 0.3, 12)
            lvl[a:b] = 0.1
            lvl[b:b + 12] = np.linspace(0.3, 0.9, 12)
            data[:, s] = lvl + 0.02 * rng.standard_normal(Tobs)
            data[a:b, s] = np.minimum(data[a:b, s], 0.2)
            data[:a, s] = np.maximum(data[:a, s], 0.26)
            data[b:, s] = np.maximum(data[b:, s], 0.26)
    hit = np.any(data[:, list(ndxS)] <= 0.25, axis=1)
    elbT0 = int(np.argmax(hit)) - p
    return bh.bh_setup(Tobs, p, 12, data, np.arange(Tobs, dtype=float), np.asarray(ndxS),
                       np.asarray(ndxO), np.ones(N), 0.25, elbT0)


def _real_bs(bh, oracle, fred):
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    return bh.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm,
                       0.25, e0)


def _flat(bh, bs, crn, NP):
    """Device CRN record: the linear blocks, uELB, then zPS padded to Ns elbT NP."""
    parts = [crn[k].ravel(order="F") for k, _ in bh.bh_crn_sizes(bs)]
    z = crn["zPS"].ravel(order="F")
    parts.append(np.concatenate([z, np.zeros(len(bs.ndxS) * bs.elbT * NP - z.size)]))
    return np.concatenate(parts)


def _run(pkg, ctx, oracle, bh, bs, B, nsweeps, NP, seed, cta_form="mirror"):
    lin = bs.lin
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=seed + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(seed)
    crns = [[bh.bh_draw_crn(rng, bs, NP) for _ in range(nsweeps)] for _ in range(B)]
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=True, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                    store_capacity=nsweeps)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_elb_ps(NP, 1)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([_flat(bh, bs, crns[c][m], NP) for m in range(nsweeps)], -1)
                     for c in range(B)], -1)
    assert flat.shape[0] == ch.crn_len
    ch.sweep(nsweeps, crn=flat, store=True)
    got = ch.get_state()
    S = ch.get_shadowrate()
    ps = ch.get_ps()
    want = []
    for c in range(B):
        st = sts[c]
        acc = []
        for m in range(nsweeps):
            prev_sqrtht = st["sqrtht"]
            st = bh.bh_sweep(st, bs, crns[c][m], elb_impl="stable", use_ps=True, cta_form=cta_form)
            acc.append(st["ps_accept"])
        st["prev_sqrtht"] = prev_sqrtht
        want.append((st, acc))
    return got, S, ps, want


def _check(oracle, bs, got, S, ps, want, tol):
    lin = bs.lin
    n_acc = 0
    for c, (st, acc) in enumerate(want):
        assert list(ps["stackAccept"][:, c]) == acc, (c, ps["stackAccept"][:, c], acc)
        n_acc += sum(1 for a in acc if a)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], 1e-2),
             "sqrtht": rel_err(got["sqrtht"][..., c], st["sqrtht"]),
             "shadowrate": rel_err(S[:, :, c], st["shadowrate"], 0.1)}
        print("chain", c, "ndxAccept", acc, e, "| PAI entries differing",
              int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        assert max(e.values()) < tol, e
        assert np.all(S[:, :, c][bs.sNaN] <= bs.ELB + 1e-12)
    assert int(ps["countAccept"].sum()) == n_acc
    return n_acc


def test_ps_toy_short_window(pkg, ctx, oracle, bh):
    """Six censored months (12 cells) where the rates glide to the ELB: most sweeps accept a
    proposal (oracle: ndxAccept 287, 228, 55, 104, 0, 264, 1, 5), one falls back to Gibbs."""
    bs = _toy_bs(bh, (114, 120), valley=True)
    got, S, ps, want = _run(pkg, ctx, oracle, bh, bs, B=4, nsweeps=2, NP=300, seed=21)
    n = _check(oracle, bs, got, S, ps, want, 1e-9)
    assert n > 0, "no proposal accepted: the test does not exercise the accept branch"


def test_ps_toy_long_window_fallback(pkg, ctx, oracle, bh):
    """Forty censored months and 2 rates: proposals rarely all land below the ELB, so the
    Gibbs fallback (:462-463) serves most sweeps."""
    bs = _toy_bs(bh, (80, 120))
    got, S, ps, want = _run(pkg, ctx, oracle, bh, bs, B=3, nsweeps=2, NP=64, seed=5)
    _check(oracle, bs, got, S, ps, want, 1e-9)


def test_ps_real_window(pkg, ctx, oracle, bh, fred):
    """Real data, jump-off 2022-08: 276 censored cells over 109 months (band width 39)."""
    bs = _real_bs(bh, oracle, fred)
    got, S, ps, want = _run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=1, NP=256, seed=8)
    _check(oracle, bs, got, S, ps, want, 1e-9)


def test_ps_mean_real_data(pkg, ctx, oracle, bh, fred):
    """The proposals' centre P^-1 b on real data, where many censored months have series above
    the ELB (observed cells of the month enter b through the residuals only): the device's
    banded factor (ccmm_chains_get_ps_mean) against the oracle's dense precision sampler at
    z = 0, at the chain's final state of a Philox sweep.  Independent of whether any proposal
    is accepted (on this window the accept branch is rare from the reference start)."""
    bs = _real_bs(bh, oracle, fred)
    lin = bs.lin
    partial = int(np.count_nonzero(np.any(bs.sNaN, axis=0) & ~np.all(bs.sNaN, axis=0)))
    assert partial > 0, "the window has no partially censored month"
    B = 2
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                    store_capacity=2, seed=91)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_elb_ps(64, 1)
    st = oracle.init_state(lin)
    ch.set_state(*[np.repeat(st[k][..., None], B, -1) for k in ("PAI", "A", "sqrtht", "h",
                                                                "sqrtPHI")])
    ch.sweep(2, store=True)
    got = ch.get_state()
    mean = ch.get_ps_mean()
    ch.close()
    N = lin.N
    for c in range(B):
        args = bh.ps_inputs(bs, got["PAI"][..., c], got["A"][..., c], got["sqrtht"][..., c])
        nmiss = int(np.count_nonzero(args[3]))
        YY = bh.precision_sampler_nan(*args, np.zeros((nmiss, 1))).reshape(N, bs.elbT, order="F")
        want = YY[bs.ndxS, :][bs.sNaN]
        have = mean[:, :bs.elbT, c][bs.sNaN]
        err = np.max(np.abs(have - want))
        print(f"chain {c}: {nmiss} censored cells, {partial} partially censored months, "
              f"max |mean diff| {err:.2e}, cells above the ELB at the mean {int(np.sum(want >= bs.ELB))}")
        assert err < 1e-8, err


def test_ps_philox_batch(pkg, ctx, oracle, bh, fred):
    """Philox stream, 32 chains, PS from the first sweep with the reference's 1000 proposals:
    status clean, censored cells below the ELB, acceptance bookkeeping consistent."""
    bs = _real_bs(bh, oracle, fred)
    lin = bs.lin
    B, nsw = 32, 3
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                    store_capacity=nsw, seed=77)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    ch.set_elb_ps(1000, 2)
    st = oracle.init_state(lin)
    ch.set_state(*[np.repeat(st[k][..., None], B, -1) for k in ("PAI", "A", "sqrtht", "h",
                                                                "sqrtPHI")])
    ch.sweep(nsw, store=True)
    assert np.all(ch.get_status() == 0)
    S = ch.get_shadowrate()
    for c in range(B):
        assert np.all(S[:, :, c][bs.sNaN] <= bs.ELB + 1e-12)
    ps = ch.get_ps()
    assert np.all(ps["stackAccept"][0] == 0)            # sweep 1: Gibbs branch
    acc = (ps["stackAccept"][1:] > 0).sum(axis=0)
    assert np.array_equal(acc, ps["countAccept"])
    assert np.all(ps["stackAccept"] <= 1000)


def test_ps_hybrid_toy(pkg, ctx, oracle, bh):
    """Hybrid model (mcmcVARhybridGibbs.m:446-483): PS proposals at every sweep with
    PAIshadow = PAI(1:Kshadow,:) and Yhatactual = Xffrlags PAIactual as intercept."""
    from oracle import ccmm_oracle_hybrid as hy
    N, p, Tobs, ndxS = 5, 2, 150, (2, 3)
    bs = _toy_bs(bh, (114, 120), valley=True)
    data = bs.lin.data
    hs = hy.hybrid_setup(Tobs, p, 12, data, np.arange(Tobs, dtype=float), np.asarray(ndxS),
                         np.ones(N), 0.25, bs.elbT0)
    lin = hs.lin
    B, nsw, NP = 4, 2, 300
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=40 + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(40)
    crns = [[hy.hybrid_draw_crn(rng, hs, NP) for _ in range(nsw)] for _ in range(B)]
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=True, model=pkg.MODEL_HYBRID,
                    Ns=len(hs.ndxS), elbTmax=hs.elbT, elb_gibbsburn=hs.gibbsburn, elb=hs.ELB,
                    store_capacity=nsw)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(hs.ndxS, None)
    ch.set_elb_slot(0, hs.elbT0, hs.sNaN)
    ch.set_elb_ps(NP, 1)
    ch.keep_missingrate(True)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])

    def flat(crn):
        parts = [crn[k].ravel(order="F") for k, _ in hy.hybrid_crn_sizes(hs)]
        z = crn["zPS"].ravel(order="F")
        parts.append(np.concatenate([z, np.zeros(len(hs.ndxS) * hs.elbT * NP - z.size)]))
        return np.concatenate(parts)

    F = np.stack([np.stack([flat(crns[c][m]) for m in range(nsw)], -1) for c in range(B)], -1)
    assert F.shape[0] == ch.crn_len
    ch.sweep(nsw, crn=F, store=True)
    got = ch.get_state()
    S = ch.get_shadowrate()
    ps = ch.get_ps()
    miss = ch.get_missingrate()          # missingrate_all (mcmcVARhybridGibbs.m:486): proposal 1
    n_acc = 0
    for c in range(B):
        st = sts[c]
        acc = []
        for m in range(nsw):
            st = hy.hybrid_sweep(st, hs, crns[c][m], use_ps=True, cta_form="mirror")
            acc.append(st["ps_accept"])
            em = rel_err(miss[m, :, :hs.elbT, c], st["missingrate"], 0.1)
            assert em < 1e-9, (c, m, em)
        n_acc += sum(1 for a in acc if a)
        assert list(ps["stackAccept"][:, c]) == acc, (c, ps["stackAccept"][:, c], acc)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], 1e-2),
             "shadowrate": rel_err(S[:, :, c], st["shadowrate"], 0.1)}
        print("hybrid chain", c, "ndxAccept", acc, e, "| PAI entries differing",
              int(np.count_nonzero(got["PAI"][..., c] != st["PAI"])))
        assert max(e.values()) < 1e-9, e
    assert n_acc > 0


@pytest.mark.parametrize("window", ["real", "toy"])
def test_ps_chol_register_window_matches_lds_kernel(pkg, ctx, oracle, bh, fred, monkeypatch, window):
    """k_ps_chol_w (register window, one wave, W <= 64) against the first-generation k_ps_chol
    (option ps_chol_lds = 1): the same band factor and forward solve in the same per-entry order, so the
    PS centre, the accepted proposals and the shadow rates of a Philox run are identical."""
    bs = _real_bs(bh, oracle, fred) if window == "real" else _toy_bs(bh, (80, 120))
    lin = bs.lin
    B, nsw = 4, 3
    outs = []
    for v1 in (1, 0):
        ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=False, model=pkg.MODEL_BLOCKHYBRID,
                        Ns=len(bs.ndxS), elbTmax=bs.elbT, elb_gibbsburn=bs.gibbsburn, elb=bs.ELB,
                        store_capacity=nsw, seed=1234, options={"ps_chol_lds": v1})
        ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
        ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
        ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
        ch.set_elb_ps(1000, 1)
        st = oracle.init_state(lin)
        ch.set_state(*[np.repeat(st[k][..., None], B, -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
        ch.sweep(nsw, store=True)
        outs.append((ch.get_ps_mean(), ch.get_ps()["stackAccept"], ch.get_shadowrate(), ch.get_status()))
        ch.close()
    (m1, a1, s1, st1), (m2, a2, s2, st2) = outs
    print(window, "accepted", int(np.count_nonzero(a2)), "max |centre diff|", float(np.nanmax(np.abs(m1 - m2))))
    assert np.all(st1 == 0) and np.all(st2 == 0)
    assert np.array_equal(a1, a2)
    np.testing.assert_array_equal(m1, m2)
    np.testing.assert_array_equal(s1, s2)
