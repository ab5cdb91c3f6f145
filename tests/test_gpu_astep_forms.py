"""The wave-parallel A-step kernel (k_astep_w, default) against the one-thread-per-regression
k_astep (CCMM_ASTEP_V1=1): mcmcVAR.m:236-254 and :259 evaluated in the same operation order
(Gram entries, left-to-right Cholesky updates, ascending substitution sums), so A, invA and the
whole chain state agree bit for bit after several real-data linear sweeps (fredblockMD20-2022-09,
N = 20, p = 12, T = 750; Philox draws, same seed)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(pkg, fred, v1, B=6, sweeps=3):
    os.environ["CCMM_ASTEP_V1"] = "1" if v1 else "0"
    try:
        mpm = pkg.model.setMinnesotaMean(fred["ncode"])
        m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
        ctx = pkg.Context(0)
        ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, seed=99)
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        st = pkg.model.initial_state(m, B)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        ch.sweep(sweeps)
        out = dict(ch.get_state())
        out["status"] = ch.get_status()
        ch.close()
        return out
    finally:
        os.environ.pop("CCMM_ASTEP_V1", None)


def test_astep_wave_form_bit_identical(pkg, fred):
    ref = _run(pkg, fred, True)
    got = _run(pkg, fred, False)
    assert not np.any(ref["status"])
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    print("k_astep_w == k_astep over", sorted(ref))
