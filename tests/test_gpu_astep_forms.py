"""The wave-parallel A-step kernel (k_astep_w, default) against the one-thread-per-regression
k_astep (CCMM_ASTEP_V1=1): mcmcVAR.m:236-254 and :259 evaluated in the same operation order
(the shared 4 x 4 Gram tiles, left-to-right Cholesky updates, ascending substitution sums, the
shared logy2 form), so A, invA and the whole chain state agree bit for bit after several sweeps:
real data (fredblockMD20-2022-09, N = 20, p = 12, T = 750; k_astep_w<20>), a synthetic 24-series
panel (k_astep_w<32>, N in 21..32) and a synthetic sample longer than 1024 months (the Gram tiles
have no sample-length limit).  Philox draws, same seed."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _synthetic(N, Nobs, seed):
    rng = np.random.default_rng(seed)
    data = np.zeros((Nobs, N))
    for t in range(1, Nobs):
        data[t] = 0.6 * data[t - 1] + rng.standard_normal(N) * (0.5 + np.arange(N) / N)
    return data, np.arange(1, Nobs + 1, dtype=float)


def _model(pkg, fred, case):
    if case == "real":
        mpm = pkg.model.setMinnesotaMean(fred["ncode"])
        return pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True), 12
    N, Nobs, p = (24, 400, 2) if case == "n24" else (6, 1100, 2)
    data, ydates = _synthetic(N, Nobs, 11 if case == "n24" else 12)
    return pkg.model.build_var(Nobs, p, 12, data, ydates, np.zeros(N), True), p


def _run(pkg, m, p, v1, B=6, sweeps=3):
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, seed=99, options={"astep_serial": int(v1)})
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(sweeps)
    out = dict(ch.get_state())
    out["status"] = ch.get_status()
    ch.close()
    return out


@pytest.mark.parametrize("case", ["real", "n24", "t1100"])
def test_astep_wave_form_bit_identical(pkg, fred, case):
    m, p = _model(pkg, fred, case)
    ref = _run(pkg, m, p, True)
    got = _run(pkg, m, p, False)
    assert not np.any(ref["status"])
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        assert np.all(np.isfinite(got[k])), k
    print(f"k_astep_w == k_astep ({case}: N = {m.N}, T = {m.T}) over", sorted(ref))
