"""The wavefront schedules of the ELB Gibbs passes (k_elb_gibbs_wf: up to 8 passes of
gibbsdrawShadowrates.m in flight, one wave each, in lock-step or with per-wave progress flags; k_elb_gibbs_oct: 8 passes in flight in one wave,
eight lanes each) reproduce the sequential kernel (k_elb_gibbs, option elb_waves = 1) bit for bit: shadow rates, every drawTruncNormal branch flag
and the whole chain state after several block-hybrid sweeps on the reference's data
(fredblockMD20-2022-09, ELB 0.25, 2022-08 jump-off: 109 censored months), with Philox draws
and with CRN-free reuse of the same seed.  Also a short censored window (2012-06 jump-off),
where fewer passes fit in flight than there are waves."""
from datetime import date

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(pkg, fred, waves, thisT, B=8, sweeps=3, oct_=0, async_=1, parts=1):
    opts = dict(elb_waves=waves, elb_oct=oct_, elb_async=async_, elb_parts=parts)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(fred["data"], ndxS, 0.25, 12)
    bm = pkg.model.build_bh(thisT, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0, True)
    m = bm.var
    ctx = pkg.Context(0)
    ch = pkg.Chains(ctx, N=m.N, p=12, T=m.T, B=B, crn=False, store_capacity=sweeps, seed=777,
                    model=pkg.MODEL_BLOCKHYBRID, Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=100,
                    elb=0.25, options=opts)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm.ndxS, bm.actual_block)
    ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.record_elb_flags(True)
    ch.sweep(sweeps, store=True)
    out = dict(ch.get_state())
    out["shadow"] = ch.get_shadowrate()
    out["flags"] = ch.get_elb_flags()
    out["status"] = ch.get_status()
    ch.close()
    return out, bm.elbT


@pytest.mark.parametrize("jump", ["last", "2012-06"])
def test_wavefront_equals_sequential(pkg, fred, jump):
    yd = np.asarray(fred["ydates"], float)            # MATLAB datenums
    jun2012 = date(2012, 6, 1).toordinal() + 366
    thisT = len(yd) if jump == "last" else int(np.nonzero(yd == jun2012)[0][0]) + 1
    ref, elbT = _run(pkg, fred, 1, thisT)
    assert not np.any(ref["status"] & ~65)
    for w in (4, 8):
        for asy in (0, 1):  # lock-step barriers / per-wave progress flags
            got, _ = _run(pkg, fred, w, thisT, async_=asy)
            for k in ref:
                np.testing.assert_array_equal(got[k], ref[k], err_msg=f"waves={w} async={asy} {k}")
    for parts in (2, 4):  # k_elb_gibbs_mp: the 8 passes over 2 / 4 CUs per chain, granule hand-offs
        got, _ = _run(pkg, fred, 8, thisT, parts=parts)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"parts={parts} {k}")
    print(f"{jump}: elbT {elbT}, {int(np.count_nonzero(ref['flags']))} flagged draws, identical for 4 and 8 waves, "
          "lock-step and asynchronous, and over 2 and 4 CUs per chain")


@pytest.mark.parametrize("parts", [2, 4])
def test_multi_cu_wavefront_one_chain(pkg, fred, parts):
    """The OOS floor's shape: ONE chain (B = 1), 101 passes over the 2022-08 window, the passes spread
    over 2 / 4 workgroups, against the sequential kernel: bit-identical."""
    thisT = len(fred["ydates"])
    ref, _ = _run(pkg, fred, 1, thisT, B=1, sweeps=2)
    got, _ = _run(pkg, fred, 8, thisT, B=1, sweeps=2, parts=parts)
    assert not np.any(got["status"] & ~65), got["status"]
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"parts={parts} {k}")


@pytest.mark.parametrize("jump,B", [("last", 19), ("2012-06", 8)])
def test_octets_equal_sequential(pkg, fred, jump, B):
    """k_elb_gibbs_oct (the kernel from B >= 384, forced with option elb_oct = 2: eight passes in flight
    inside one wave, eight lanes per pass, octet sums in wave_sum_dpp's tree order) against the sequential one-wave kernel
    (elb_oct = 0, elb_waves = 1): shadow rates, every drawTruncNormal branch flag and the chain
    state bit for bit."""
    yd = np.asarray(fred["ydates"], float)
    jun2012 = date(2012, 6, 1).toordinal() + 366
    thisT = len(yd) if jump == "last" else int(np.nonzero(yd == jun2012)[0][0]) + 1
    ref, elbT = _run(pkg, fred, 1, thisT, B=B)
    got, _ = _run(pkg, fred, 8, thisT, B=B, oct_=2)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"octets {k}")
    print(f"{jump}: elbT {elbT}, B {B}: octet kernel identical ({int(np.count_nonzero(ref['flags']))} flagged draws)")
