"""The partitioned SV smoother split over two workgroups per chain (default for 32 < B <= 128:
phase A over 2 x 8 waves, then phases B + C with the serial separator pass redone by each
workgroup) and over four (default for B <= 32: 4 x 4 waves, one per SIMD) against the
one-workgroup launch (option sv_nwg = 1): the same segments, separators and operation order, so h,
eta, sqrtht and the whole chain state agree bit for bit after several real-data linear sweeps
(fredblockMD20-2022-09, N = 20, p = 12; Philox draws).  T = 750 has 16 segments (one per wave);
the short sample (T = 72) has 9, so some workgroups run one segment or none besides their copy of
the separator pass."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(pkg, fred, nwg, thisT, B=6, sweeps=3):
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    m = pkg.model.build_var(thisT, 12, 12, fred["data"], fred["ydates"], mpm, True)
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, seed=7, options={"sv_nwg": nwg})
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(sweeps)
    out = dict(ch.get_state())
    out["status"] = ch.get_status()
    ch.close()
    return out


@pytest.mark.parametrize("short", [False, True])
@pytest.mark.parametrize("nwg", [2, 4])
def test_sv_split_workgroups_bit_identical(pkg, fred, short, nwg):
    thisT = 12 + 12 + 60 if short else len(fred["ydates"])
    ref = _run(pkg, fred, 1, thisT)
    got = _run(pkg, fred, nwg, thisT)
    assert not np.any(ref["status"])
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    print(f"SV nwg={nwg} == nwg=1 over", sorted(ref), "T =", thisT)


def test_sv_mfma_products_match_fma_pass(pkg, fred):
    """Phase A's block products on MFMA (option sv_mfma = 1, the default at N = 20) against the FMA pass
    (sv_mfma = 0): the same sampler in another accumulation order, so not bit-identical -- agreement to
    rounding.  One real-data linear sweep from the same state and streams (N = 20, T = 750), every
    workgroup layout: h and sqrtht within 1e-12 relative, the KSC indicators identical."""
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    ctx = pkg.Context(0)
    outs = {}
    for mf in (0, 1):
        ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=6, crn=False, seed=7, options={"sv_mfma": mf})
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        st = pkg.model.initial_state(m, 6)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        ch.sweep(1)
        outs[mf] = (ch.get_state(), ch.get_kai(), ch.get_status())
        ch.close()
    (s0, k0, st0), (s1, k1, st1) = outs[0], outs[1]
    assert not np.any(st0) and not np.any(st1)
    np.testing.assert_array_equal(k0, k1)
    for k in ("h", "sqrtht"):
        err = np.max(np.abs(s1[k] - s0[k]) / np.maximum(np.abs(s0[k]), 1.0))
        print(f"sv_mfma 1 vs 0: {k} max rel {err:.2e}")
        assert err < 1e-12, (k, err)
