"""GPU parity of the predictive density computed inside the chain set
(ccmm_chains_set_fcst: every stored sweep forecasts on the device from the chain's own
draw and data) against the oracle restatements:

  * block hybrid: oracle/ccmm_oracle_fcst.fcst_draw_bh (mcmcVARshadowrateBlockHybrid.m:
    550-625 as written, dense companion on K + Nyields p states), two real-data vintages
    of different T / elbT in one chain set (an ELB-era vintage with three yields at the
    ELB, a 2017 vintage with none), two chains each;
  * linear: oracle/ccmm_oracle_fcst.fcst_draw (mcmcVAR.m:298-381).

The forecast block is checked on the GPU's own post-sweep state (PAI, invA, Vol_states,
sqrtPHI, the shadow-rate Y), so its tolerance does not inherit the sweep's (the sweep
itself: test_gpu_bh.py / test_gpu_parity.py).  Tolerances as tests/test_gpu_fcst.py:
paths 1e-9 in |Δ| / max(|x|, 1); scores 1e-9, 1e-8 with three series at the ELB
(trivariate mvncdf)."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

H, ND = 12, 5


@pytest.fixture(scope="module")
def F():
    from oracle import ccmm_oracle_fcst
    return ccmm_oracle_fcst


def _bh_vintages(pkg, fred, offsets):
    d = fred
    p = 12
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    out = []
    for thisT in offsets:
        bm = pkg.model.build_bh(thisT, p, 12, d["data"], d["ydates"], ndxS, ndxO, mpm, 0.25, e0)
        yr = pkg.samplers.realized_values(d["data"], thisT, H, ndxS, 0.25)
        out.append((thisT, bm, yr))
    return out, ndxS, ndxY


def test_bh_chain_fcst_two_vintages(pkg, ctx, fred, F):
    p = 12
    nT = len(fred["ydates"])
    vint, ndxS, ndxY = _bh_vintages(pkg, fred, [585 + p + 1 + 40, nT - 60])
    C = 2
    B = C * len(vint)
    Tmax = max(v[1].var.T for v in vint)
    elbTmax = max(v[1].elbT for v in vint)
    m0 = vint[0][1]
    ch = pkg.Chains(ctx, N=m0.var.N, p=p, T=Tmax, B=B, ndata=len(vint), crn=True,
                    model=pkg.MODEL_BLOCKHYBRID, Ns=len(ndxS), elbTmax=elbTmax, elb_gibbsburn=20,
                    elb=0.25, store_capacity=2)
    for s, (thisT, bm, yr) in enumerate(vint):
        m = bm.var
        ch.set_data(s, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(m0.ndxS, m0.actual_block)
    yields = np.zeros(m0.var.N, bool)
    yields[ndxY] = True
    ch.set_fcst(H, ND, yields, keep_paths=True)
    slots = np.repeat(np.arange(len(vint)), C)
    ch.set_slots(slots)
    init = {k: np.zeros(sh) for k, sh in (("PAI", (m0.var.K, m0.var.N, B)), ("A", (m0.var.N,) * 2 + (B,)),
                                           ("sqrtht", (Tmax, m0.var.N, B)), ("h", (Tmax, m0.var.N, B)),
                                           ("sqrtPHI", (m0.var.N,) * 2 + (B,)))}
    for s, (thisT, bm, yr) in enumerate(vint):
        ch.set_elb_slot(s, bm.elbT0, bm.sNaN)
        ch.set_fcst_slot(s, yr[:, 0])
        st = pkg.model.initial_state(bm.var, C)
        T = bm.var.T
        for k in init:
            v = st[k]
            if k in ("sqrtht", "h"):
                pad = np.ones((Tmax - T,) + v.shape[1:]) if k == "sqrtht" else np.zeros((Tmax - T,) + v.shape[1:])
                v = np.concatenate([v, pad], axis=0)
            init[k][..., s * C:(s + 1) * C] = v
    ch.set_state(init["PAI"], init["A"], init["sqrtht"], init["h"], init["sqrtPHI"])
    rng = np.random.default_rng(11)
    crn = ch.draw_crn(rng, 2)
    ch.sweep(1, crn=crn[:, :1], store=False)
    ch.sweep(1, crn=crn[:, 1:], store=True)
    st = ch.get_state()
    X, Y = ch.get_xy()
    fc = ch.get_fcst(paths=True)
    assert fc["M"] == 1 and not fc["warn_mvncdf"]
    off, n, _ = ch.crn_layout()["FCST"]
    N = m0.var.N
    nat_seen = set()
    for c in range(B):
        thisT, bm, yr = vint[slots[c]]
        T = bm.var.T
        data_v = fred["data"][:thisT]
        Xj = F.bh_jumpoff(Y[:T, :, c], data_v, p, yields)
        seg = crn[off:off + n, 1, c]
        svz = seg[:N * H * ND].reshape(N, H * ND, order="F")
        z = seg[N * H * ND:].reshape(N, H, ND, order="F")
        fY, sc = F.fcst_draw_bh(st["PAI"][..., c], st["invA"][..., c], st["h"][T - 1, :, c],
                                st["sqrtPHI"][..., c], Xj, yr[:, 0], yields, m0.actual_block, 0.25,
                                svz, z)
        got = fc["paths"][..., 0, c]
        e = rel_err(got, fY, 1.0)
        assert e < 1e-9, (c, e)
        # fcstYdraws: yields floored at the ELB after the simulation (:696-700)
        fYc = fY.copy()
        fYc[yields] = np.maximum(fYc[yields], 0.25)
        assert rel_err(fc["paths_censored"][..., 0, c], fYc, 1.0) < 1e-9
        assert rel_err(fc["fYsum"][..., c], fY.sum(axis=2), 1.0) < 1e-9
        nat = int(np.sum(yr[yields, 0] <= 0.25))
        nat_seen.add(nat)
        gsc = fc["scores"][:, 0, :, c]          # Nd x 4
        tol = 1e-8 if nat == 3 else 1e-9
        for k_dev, k_or in ((1, 0), (2, 1), (3, 2)):
            e = rel_err(gsc[:, k_dev], sc[k_or], 1.0)
            assert e < tol, (c, k_dev, e)
    assert nat_seen == {0, 3}, nat_seen


def test_linear_chain_fcst_matches_oracle(pkg, ctx, oracle, fred, F):
    """Linear chain set (configs[1] data, jump-off 2020-03: the funds rate realized at the ELB
    in 2020-04): stored sweeps carry fcstYdraws, fcstYcensorDraws, the zero-shock
    mean path and the four score draws, each equal to fcst_draw on the GPU's state."""
    p = 12
    thisT = len(fred["ydates"]) - 29
    ndxS, _, ndxY = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    m = pkg.model.build_var(thisT, p, 12, fred["data"], fred["ydates"], mpm, True)
    yr = pkg.samplers.realized_values(fred["data"], thisT, H, ndxS, 0.25)
    B = 3
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=True, store_capacity=2)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    yields = np.zeros(m.N, bool)
    yields[ndxY] = True
    ch.set_fcst(H, ND, yields, keep_paths=True)
    ch.set_fcst_slot(0, yr[:, 0])
    st0 = pkg.model.initial_state(m, B)
    ch.set_state(st0["PAI"], st0["A"], st0["sqrtht"], st0["h"], st0["sqrtPHI"])
    crn = ch.draw_crn(np.random.default_rng(5), 2)
    ch.sweep(2, crn=crn, store=True)
    st = ch.get_state()
    fc = ch.get_fcst(paths=True)
    assert fc["M"] == 2
    off, n, _ = ch.crn_layout()["FCST"]
    N = m.N
    for c in range(B):
        seg = crn[off:off + n, 1, c]
        svz = seg[:N * H * ND].reshape(N, H * ND, order="F")
        z = seg[N * H * ND:].reshape(N, H, ND, order="F")
        fY, fYc, yhat, sc = F.fcst_draw(st["PAI"][..., c], st["invA"][..., c], st["h"][-1, :, c],
                                        st["sqrtPHI"][..., c], m.Xjumpoff, yr[:, 0], yields, 0.25,
                                        svz, z)
        assert rel_err(fc["paths"][..., 1, c], fY, 1.0) < 1e-9
        assert rel_err(fc["paths_censored"][..., 1, c], fYc, 1.0) < 1e-9
        e = rel_err(fc["scores"][:, 1, :, c].T, sc, 1.0)
        assert e < 1e-8, (c, e)
    # running sums cover both kept draws
    assert rel_err(fc["fYsum"], fc["paths"].sum(axis=(2, 3)), 1.0) < 1e-12
    # get_fcst resets the records
    assert ch.fcst_stored() == 0
