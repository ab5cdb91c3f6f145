"""BASELINE.json configs[4] at its full shape: the block-hybrid shadow-rate
sweep on the synthetic S120 panel, N = 120, p = 12, T = 750, K = 1441 (KP = 1472), Ns = 4
shadow rates, elbT = 114, every block on the large path (ccmm_big.hip multi-equation Gram
at N = 120 with two design slabs, blocked MFMA Cholesky of 1472 x 1472 systems, per-chain
solve; ccmm_bign.hip A / SV / PHI; the N > 64 ELB kernels).

(a) CRN: one sweep of two chains against the oracle's bh_sweep with CTAsys in the
    weighted-SYRK form (oracle.cta_sys_syrk: the kron form would materialise 1 GB per
    equation) and the stable ELB form.  Tolerances as test_gpu_bign.py (units of
    max(|x|, sd_post)); KSC indicators and truncated-normal branch flags bit-exact.
(b) Philox: four chains, three sweeps: finite draws, censored shadow rates at or below
    the ELB, status 0.
"""
import numpy as np
import pytest

from conftest import rel_err
from helpers import bh_crn_flat, random_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s120(pkg, oracle):
    from oracle import ccmm_oracle_bh as bh
    d = pkg.synthetic.s120()
    ndxS, ndxO, _ = oracle.set_shadow_yields(d["ncode"], 0.25)
    e0 = oracle.elb_t0(d["data"], ndxS, 0.25, 12)
    bs = bh.bh_setup(len(d["ydates"]), 12, 12, d["data"], d["ydates"], ndxS, ndxO,
                     np.ones(d["data"].shape[1]), 0.25, e0)
    assert (bs.lin.N, bs.lin.K, bs.lin.T, len(bs.ndxS)) == (120, 1441, 750, 4)
    return d, bs


def _chain_set(pkg, ctx, bs, B, crn):
    lin = bs.lin
    ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=B, crn=crn, store_capacity=4,
                    model=pkg.MODEL_BLOCKHYBRID, Ns=len(bs.ndxS), elbTmax=bs.elbT,
                    elb_gibbsburn=bs.gibbsburn, elb=bs.ELB, seed=20230101)
    ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
    ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
    ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
    return ch


def test_s120_bh_sweep_crn(pkg, ctx, oracle, s120):
    from oracle import ccmm_oracle_bh as bh
    _, bs = s120
    lin = bs.lin
    B = 2
    sts = []
    for c in range(B):
        st = random_state(oracle, lin, seed=50 + c)
        st["X"], st["Y"] = lin.X.copy(), lin.Y.copy()
        sts.append(st)
    rng = np.random.default_rng(7)
    crns = [bh.bh_draw_crn(rng, bs) for _ in range(B)]
    ch = _chain_set(pkg, ctx, bs, B, crn=True)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
    ch.record_elb_flags(True)
    flat = np.stack([bh_crn_flat(bh, crns[c], bs)[:, None] for c in range(B)], -1)
    ch.sweep(1, crn=flat)
    got = ch.get_state()
    S = ch.get_shadowrate()
    kai = ch.get_kai()
    flags = ch.get_elb_flags()
    status = ch.get_status()
    ch.close()
    assert not status.any(), status
    for c in range(B):
        prev = sts[c]["sqrtht"]
        want = bh.bh_sweep(sts[c], bs, crns[c], return_flags=True, elb_impl="stable", cta_form="syrk")
        Xs = [bs.Xactual if bs.actualrateBlock[j] else sts[c]["X"] for j in range(lin.N)]
        _, _, sd = oracle.cta_sys_syrk(sts[c]["Y"], Xs, lin.N, lin.K, lin.T, want["A"], want["sqrtht"],
                                       lin.iVdiag, lin.iVb, want["PAI"], np.zeros((lin.K, lin.N)),
                                       return_sd=True)
        e = {"PAI": rel_err(got["PAI"][..., c], want["PAI"], sd),
             "A": rel_err(got["A"][..., c], want["A"], oracle.a_step_sd(want["RESID"], prev)),
             "sqrtht": rel_err(got["sqrtht"][..., c], want["sqrtht"]),
             "sqrtPHI": rel_err(got["sqrtPHI"][..., c], want["sqrtPHI"], 1e-3),
             "shadowrate": rel_err(S[:, :bs.elbT, c], want["shadowrate"], 0.1)}
        print("S120 chain", c, {k: f"{v:.2e}" for k, v in e.items()})
        np.testing.assert_array_equal(kai[..., c], want["kai"])                 # KSC: bit-exact
        np.testing.assert_array_equal(flags[:, :bs.elbT, :, c], want["elb_flags_stable"])
        assert np.all(S[:, :bs.elbT, c][bs.sNaN] <= bs.ELB + 1e-12)
        assert max(e.values()) < 1e-10, e   # measured 1.5e-11 (r03)


def test_s120_philox_property(pkg, ctx, s120):
    _, bs = s120
    lin = bs.lin
    B = 4
    ch = _chain_set(pkg, ctx, bs, B, crn=False)
    st = pkg.model.initial_state(lin, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(2, store=False)
    ch.sweep(1, store=True)
    S = ch.get_shadowrate()
    dr = ch.get_draws()
    status = ch.get_status()
    ch.close()
    assert not status.any(), status
    for k, v in dr.items():
        assert np.all(np.isfinite(v)), k
    for c in range(B):
        assert np.all(S[:, :bs.elbT, c][bs.sNaN] <= bs.ELB + 1e-12)
        assert np.all(np.isfinite(S[:, :bs.elbT, c]))
    assert np.std(dr["PAI_all"][-1, 1, 0, :]) > 0   # chains differ
