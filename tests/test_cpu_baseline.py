"""The compiled CPU baseline (oracle/cpu_sweep.cpp: the linear sweep of mcmcVAR.m:211-274 as written,
kron-materialised CTA with the explicit inverse, OpenBLAS, one thread) against the numpy oracle on the
same common random numbers: the same sweep up to summation order (the SV block in the time-ordered
block-Cholesky convention, oracle.sv_draw_sequential, which the binary implements)."""
import numpy as np
import pytest

from conftest import rel_err


def _oracle_sweep(O, st, su, crn):
    """oracle.linear_sweep with the time-ordered SV sampler (the binary's convention)."""
    N, K = su.N, su.K
    PAI, _, sd = O.cta(su.Y, su.X, N, K, st["A"], st["sqrtht"], su.iVdiag, su.iVb, st["PAI"], crn["zPAI"],
                       return_sd=True)
    RESID = su.Y - su.X @ PAI
    A, _ = O.a_step(RESID, st["sqrtht"], crn["zA"])
    logy2 = np.log((RESID @ A.T) ** 2 + su.logy2offset)
    kai = O.ksc_indicators(logy2.T, st["h"].T, crn["uSV"])
    obs = logy2.T - O.KSC_MEAN[kai - 1]
    ir = 1.0 / O.KSC_VAR[kai - 1]
    D, b, Q = O.sv_precision(obs, ir, st["sqrtPHI"], su.Vol_0mean, su.Vol_0vcvsqrt)
    x = O.sv_draw_sequential(D, b, Q, crn["zSV"])
    h = x[1:]
    sqrtPHI, _ = O.phi_iw(x[1:] - x[:-1], su.sPHI, crn["zPHI"])
    return dict(PAI=PAI, A=A, h=h, sqrtht=np.exp(h / 2), sqrtPHI=sqrtPHI, kai=kai), sd


@pytest.mark.parametrize("form", ["kron", "syrk"])
@pytest.mark.parametrize("shape", ["toy", "real"])
def test_cpu_sweep_matches_oracle(oracle, fred, tmp_path, shape, form):
    """Both CPU lines: CTA as written (kron) and the algorithmic weighted-SYRK form (bench-syrk)."""
    from helpers import random_state
    from oracle import cpu_baseline as CB
    O = oracle
    mpm = O.set_minnesota_mean(fred["ncode"])
    if shape == "toy":
        sel = [0, 4, 14, 17]
        su = O.var_setup(80, 2, 12, fred["data"][-80:, sel], fred["ydates"][-80:], mpm[sel], True)
    else:
        su = O.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    st = random_state(O, su, seed=5)
    crn = O.draw_crn(np.random.default_rng(6), su.N, su.K, su.T, su.dPHI)
    got = CB.crn_sweep(su, st, crn, tmp_path, form=form)
    want, sd = _oracle_sweep(O, st, su, crn)
    np.testing.assert_array_equal(got["kai"], want["kai"])
    e = {"PAI": rel_err(got["PAI"], want["PAI"], sd), "A": rel_err(got["A"], want["A"], 1.0),
         "sqrtht": rel_err(got["sqrtht"], want["sqrtht"]), "sqrtPHI": rel_err(got["sqrtPHI"], want["sqrtPHI"], 1e-3)}
    print(shape, form, e)
    assert max(e.values()) < 1e-7, e


def test_cpu_sweep_bench_mode(oracle, fred, tmp_path):
    from oracle import cpu_baseline as CB
    O = oracle
    mpm = O.set_minnesota_mean(fred["ncode"])
    sel = [0, 4, 14, 17]
    su = O.var_setup(80, 2, 12, fred["data"][-80:, sel], fred["ydates"][-80:], mpm[sel], True)
    CB.write_state(tmp_path / "s.bin", su, O.init_state(su))
    n, el = CB.bench_result(CB.bench_process(tmp_path / "s.bin", 0.2, 1), 60)
    assert n >= 1 and el >= 0.2


def _oracle_bh_sweep(O, BH, st, bs, crn):
    """oracle.ccmm_oracle_bh.bh_sweep (kron CTAsys, gibbsdrawShadowrates as written) with the
    time-ordered SV sampler (the binary's convention)."""
    lin = bs.lin
    N, K, T = lin.N, lin.K, lin.T
    X, Y = st["X"], st["Y"]
    XX = np.empty((T, K, N))
    XX[:, :, bs.actualrateBlock] = bs.Xactual[:, :, None]
    XX[:, :, ~bs.actualrateBlock] = X[:, :, None]
    PAI, _, sd = O.cta_sys(Y, XX, N, K, T, st["A"], st["sqrtht"], lin.iVdiag, lin.iVb, st["PAI"], crn["zPAI"],
                           return_sd=True)
    RESID = np.stack([Y[:, j] - XX[:, :, j] @ PAI[:, j] for j in range(N)], axis=1)
    A, invA = O.a_step(RESID, st["sqrtht"], crn["zA"])
    logy2 = np.log((RESID @ A.T) ** 2 + lin.logy2offset)
    kai = O.ksc_indicators(logy2.T, st["h"].T, crn["uSV"])
    obs = logy2.T - O.KSC_MEAN[kai - 1]
    ir = 1.0 / O.KSC_VAR[kai - 1]
    D, b, Q = O.sv_precision(obs, ir, st["sqrtPHI"], lin.Vol_0mean, lin.Vol_0vcvsqrt)
    x = O.sv_draw_sequential(D, b, Q, crn["zSV"])
    h = x[1:]
    sqrtht = np.exp(h / 2)
    sqrtPHI, _ = O.phi_iw(x[1:] - x[:-1], lin.sPHI, crn["zPHI"])
    C, Psi, SVol, Yhatactual = BH.elb_state_space(bs, PAI, invA, sqrtht)
    sr = O.gibbsdraw_shadowrates(Y[bs.elbT0:, :].T, bs.X0, Yhatactual, bs.ndxSmask, bs.sNaN, lin.p, C, Psi, SVol,
                                 bs.ELB, 1, bs.gibbsburn, crn["uELB"])[:, :, 0]
    return dict(PAI=PAI, A=A, h=h, sqrtht=sqrtht, sqrtPHI=sqrtPHI, kai=kai, shadowrate=sr), sd


@pytest.mark.parametrize("form", ["kron", "syrk"])
@pytest.mark.parametrize("shape", ["toy", "real"])
def test_cpu_sweep_blockhybrid_matches_oracle(oracle, fred, tmp_path, shape, form):
    """The compiled block-hybrid sweep (kron CTAsys, gibbsdrawShadowrates as written with dgeqrf, 101
    Gibbs passes) against the numpy oracle on the same common random numbers."""
    from helpers import random_state, synth_bh_data
    from oracle import ccmm_oracle_bh as BH
    from oracle import cpu_baseline as CB
    O = oracle
    if shape == "toy":
        N, p, Tobs, ndxS, ndxO = 5, 2, 150, (2, 3), (4,)
        data = synth_bh_data(N, p, Tobs, elb_window=(100, 130), ndxS=ndxS, seed=4)
        hit = np.any(data[:, list(ndxS)] <= 0.25, axis=1)
        bs = BH.bh_setup(Tobs, p, 12, data, np.arange(Tobs, dtype=float), np.asarray(ndxS), np.asarray(ndxO),
                         np.ones(N), 0.25, int(np.argmax(hit)) - p)
        bs.gibbsburn = 10
        st = random_state(O, bs.lin, seed=9)
    else:
        ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
        mpm = O.set_minnesota_mean(fred["ncode"])
        e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
        bs = BH.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
        bs.gibbsburn = 3   # the pass loop is the same code for every pass; keep the numpy side short
        st = random_state(O, bs.lin, seed=9)   # (the reference initialisation's CTA sits at cond ~1e13)
    st["X"], st["Y"] = bs.lin.X.copy(), bs.lin.Y.copy()
    crn = BH.bh_draw_crn(np.random.default_rng(7), bs)
    got = CB.crn_sweep(bs.lin, st, crn, tmp_path, bs, form=form)
    want, sd = _oracle_bh_sweep(O, BH, st, bs, crn)
    np.testing.assert_array_equal(got["kai"], want["kai"])
    e = {"PAI": rel_err(got["PAI"], want["PAI"], sd), "A": rel_err(got["A"], want["A"], 1.0),
         "sqrtht": rel_err(got["sqrtht"], want["sqrtht"]), "sqrtPHI": rel_err(got["sqrtPHI"], want["sqrtPHI"], 1e-3),
         "shadowrate": rel_err(got["shadowrate"], want["shadowrate"], 0.1)}
    print(shape, form, e)
    assert max(e.values()) < 1e-7, e


def test_cpu_sweep_blockhybrid_bench_mode(oracle, fred, tmp_path):
    from oracle import ccmm_oracle_bh as BH
    from oracle import cpu_baseline as CB
    O = oracle
    ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
    mpm = O.set_minnesota_mean(fred["ncode"])
    e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
    bs = BH.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
    st = BH.bh_init_state(bs)
    CB.write_state(tmp_path / "s.bin", bs.lin, st, bs)
    for form in ("kron", "syrk"):
        n, el = CB.bench_result(CB.bench_process(tmp_path / "s.bin", 0.5, 1, form=form), 120)
        assert n >= 1 and el >= 0.5
