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


@pytest.mark.parametrize("shape", ["toy", "real"])
def test_cpu_sweep_matches_oracle(oracle, fred, tmp_path, shape):
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
    got = CB.crn_sweep(su, st, crn, tmp_path)
    want, sd = _oracle_sweep(O, st, su, crn)
    np.testing.assert_array_equal(got["kai"], want["kai"])
    e = {"PAI": rel_err(got["PAI"], want["PAI"], sd), "A": rel_err(got["A"], want["A"], 1.0),
         "sqrtht": rel_err(got["sqrtht"], want["sqrtht"]), "sqrtPHI": rel_err(got["sqrtPHI"], want["sqrtPHI"], 1e-3)}
    print(shape, e)
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
