"""Vintage batch: the goVAR* parfor over quasi-real-time vintages
(goVAR.m:242, goVARshadowrateBlockHybrid.m:258) becomes one device chain set whose
chains are bound to data slots of different lengths T.  Each chain is checked
against the oracle sweep of its own vintage, common random numbers per chain (a
chain of a shorter vintage reads the leading part of each CRN block, the MATLAB
column-major arrays of its own shapes)."""
import numpy as np
import pytest

from conftest import rel_err
from helpers import random_state

pytestmark = pytest.mark.gpu


def _pad_flat(sizes_max, crn):
    out = []
    for name, shape in sizes_max:
        blk = np.zeros(int(np.prod(shape)))
        a = crn[name].ravel(order="F")
        blk[:a.size] = a
        out.append(blk)
    return np.concatenate(out)


def _pad_rows(a, T, fill):
    out = np.full((T,) + a.shape[1:], fill)
    out[:a.shape[0]] = a
    return out


def _stack_state(sts, Tmax):
    return [np.stack([s["PAI"] for s in sts], -1), np.stack([s["A"] for s in sts], -1),
            np.stack([_pad_rows(s["sqrtht"], Tmax, 1.0) for s in sts], -1),
            np.stack([_pad_rows(s["h"], Tmax, 0.0) for s in sts], -1),
            np.stack([s["sqrtPHI"] for s in sts], -1)]


def test_linear_vintages_crn(pkg, ctx, oracle, fred):
    """Three vintages (jump-offs 2019-04, 2021-12, 2022-08: T = 710, 742, 750) x two
    chains each, interleaved over the slots; one CRN sweep per chain."""
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    nT = len(fred["ydates"])
    thisTs = [nT - 40, nT - 8, nT]
    sus = [oracle.var_setup(t, 12, 12, fred["data"], fred["ydates"], mpm, True) for t in thisTs]
    Tmax = max(su.T for su in sus)
    assert sorted({su.T for su in sus}) == [710, 742, 750]
    slots = [0, 1, 2, 2, 1, 0]
    B = len(slots)
    su0 = sus[-1]
    ch = pkg.Chains(ctx, N=su0.N, p=12, T=Tmax, B=B, ndata=3, crn=True)
    for s, t in enumerate(thisTs):
        m = pkg.model.build_var(t, 12, 12, fred["data"], fred["ydates"], mpm, True)
        ch.set_data(s, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_slots(slots)
    sts = [random_state(oracle, sus[slots[c]], seed=300 + c) for c in range(B)]
    ch.set_state(*_stack_state(sts, Tmax))
    rng = np.random.default_rng(31)
    crns = [oracle.draw_crn(rng, su0.N, su0.K, sus[slots[c]].T, su0.dPHI) for c in range(B)]
    sizes_max = oracle.crn_sizes(su0.N, su0.K, Tmax, su0.dPHI)
    flat = np.stack([_pad_flat(sizes_max, crns[c])[:, None] for c in range(B)], -1)
    assert flat.shape[0] == ch.crn_len
    ch.sweep(1, crn=flat)
    got = ch.get_state()
    for c in range(B):
        su = sus[slots[c]]
        st0 = sts[c]
        st = oracle.linear_sweep(st0, su, crns[c], cta_form="mirror")
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, st0["A"], st0["sqrtht"], su.iVdiag, su.iVb,
                              st0["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], sd),
             "A": rel_err(got["A"][..., c], st["A"], oracle.a_step_sd(st["RESID"], st0["sqrtht"])),
             "sqrtht": rel_err(got["sqrtht"][:su.T, :, c], st["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], st["sqrtPHI"], 1e-3)}
        print("chain", c, "T", su.T, e)
        assert max(e.values()) < 1e-9, e


def test_bh_vintages_crn(pkg, ctx, oracle, fred):
    """Block-hybrid vintages with different ELB windows (elbT = 125, 157, 165): one CRN
    sweep per chain, shadow rates and rebuilt X/Y per vintage."""
    from oracle import ccmm_oracle_bh as bh
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    nT = len(fred["ydates"])
    thisTs = [nT - 40, nT - 8, nT]
    bss = [bh.bh_setup(t, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
           for t in thisTs]
    assert [b.elbT for b in bss] == [125, 157, 165]
    Tmax = max(b.lin.T for b in bss)
    elbTmax = max(b.elbT for b in bss)
    slots = [2, 0, 1]
    B = len(slots)
    lin0 = bss[-1].lin
    ch = pkg.Chains(ctx, N=lin0.N, p=12, T=Tmax, B=B, ndata=3, crn=True, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(ndxS), elbTmax=elbTmax, elb_gibbsburn=100, elb=0.25)
    for s, b in enumerate(bss):
        L = b.lin
        ch.set_data(s, L.Y, L.X, L.iVdiag, L.iVb, L.sPHI, L.Vol_0mean, L.Vol_0vcvsqrt)
    ch.set_slots(slots)
    ch.set_elb_model(bss[0].ndxS, bss[0].actualrateBlock)
    for s, b in enumerate(bss):
        ch.set_elb_slot(s, b.elbT0, b.sNaN)
    sts = []
    for c in range(B):
        L = bss[slots[c]].lin
        st = random_state(oracle, L, seed=400 + c)
        st["X"], st["Y"] = L.X.copy(), L.Y.copy()
        sts.append(st)
    ch.set_state(*_stack_state(sts, Tmax))
    rng = np.random.default_rng(41)
    crns = [bh.bh_draw_crn(rng, bss[slots[c]]) for c in range(B)]
    sizes_max = oracle.crn_sizes(lin0.N, lin0.K, Tmax, lin0.dPHI) + [
        ("uELB", (len(ndxS), elbTmax, 101))]
    flat = np.stack([_pad_flat(sizes_max, crns[c])[:, None] for c in range(B)], -1)
    assert flat.shape[0] == ch.crn_len
    ch.sweep(1, crn=flat)
    got = ch.get_state()
    S = ch.get_shadowrate()
    X, Y = ch.get_xy()
    for c in range(B):
        b = bss[slots[c]]
        T = b.lin.T
        st = bh.bh_sweep(sts[c], b, crns[c], elb_impl="stable", cta_form="mirror")
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], 1.0),
             "sqrtht": rel_err(got["sqrtht"][:T, :, c], st["sqrtht"]),
             "shadowrate": rel_err(S[:, :b.elbT, c], st["shadowrate"], 0.1),
             "X": rel_err(X[:T, :, c], st["X"], 0.1), "Y": rel_err(Y[:T, :, c], st["Y"], 0.1)}
        print("chain", c, "T", T, "elbT", b.elbT, e)
        assert max(e.values()) < 1e-9, e


def test_bh_vintage_range_crn(pkg, ctx, oracle, fred):
    """Every eighth vintage of the configs[3] OOS set (goVARshadowrateBlockHybrid.m:127, jump-offs
    after 2008-12) plus the last, one chain each on one chain set: ELB windows from two censored
    months (the first vintages) to 165, vintages after the 2015 lift-off with uncensored months
    inside the window; one CRN sweep per chain against its vintage's oracle sweep."""
    from oracle import ccmm_oracle_bh as bh
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
    Tj = list(np.flatnonzero(fred["ydates"] > pkg.samplers.datenum(2008, 12, 1)) + 1)
    assert len(Tj) == 164
    thisTs = Tj[::8] + ([Tj[-1]] if (len(Tj) - 1) % 8 else [])
    bss = [bh.bh_setup(int(t), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0) for t in thisTs]
    elbTs = [b.elbT for b in bss]
    assert min(elbTs) <= 10 and max(elbTs) == 165
    Tmax = max(b.lin.T for b in bss)
    elbTmax = max(elbTs)
    B = len(bss)
    lin0 = bss[-1].lin
    ch = pkg.Chains(ctx, N=lin0.N, p=12, T=Tmax, B=B, ndata=B, crn=True, model=pkg.MODEL_BLOCKHYBRID,
                    Ns=len(ndxS), elbTmax=elbTmax, elb_gibbsburn=100, elb=0.25)
    for s, b in enumerate(bss):
        L = b.lin
        ch.set_data(s, L.Y, L.X, L.iVdiag, L.iVb, L.sPHI, L.Vol_0mean, L.Vol_0vcvsqrt)
    ch.set_slots(list(range(B)))
    ch.set_elb_model(bss[0].ndxS, bss[0].actualrateBlock)
    for s, b in enumerate(bss):
        ch.set_elb_slot(s, b.elbT0, b.sNaN)
    sts = []
    for c, b in enumerate(bss):
        st = random_state(oracle, b.lin, seed=500 + c)
        st["X"], st["Y"] = b.lin.X.copy(), b.lin.Y.copy()
        sts.append(st)
    ch.set_state(*_stack_state(sts, Tmax))
    rng = np.random.default_rng(51)
    crns = [bh.bh_draw_crn(rng, b) for b in bss]
    sizes_max = oracle.crn_sizes(lin0.N, lin0.K, Tmax, lin0.dPHI) + [("uELB", (len(ndxS), elbTmax, 101))]
    flat = np.stack([_pad_flat(sizes_max, crns[c])[:, None] for c in range(B)], -1)
    ch.sweep(1, crn=flat)
    got = ch.get_state()
    S = ch.get_shadowrate()
    status = ch.get_status()
    ch.close()
    worst = 0.0
    for c, b in enumerate(bss):
        T = b.lin.T
        st = bh.bh_sweep(sts[c], b, crns[c], elb_impl="stable", cta_form="mirror")
        e = {"PAI": rel_err(got["PAI"][..., c], st["PAI"], 1.0),
             "sqrtht": rel_err(got["sqrtht"][:T, :, c], st["sqrtht"]),
             "shadowrate": rel_err(S[:, :b.elbT, c], st["shadowrate"], 0.1)}
        worst = max(worst, max(e.values()))
        assert max(e.values()) < 1e-9, (thisTs[c], b.elbT, e)
    print(f"{B} vintages (elbT {min(elbTs)}..{max(elbTs)}), worst rel err {worst:.2e}, status {set(status.tolist())}")
