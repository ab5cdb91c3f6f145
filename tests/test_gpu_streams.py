"""Schedules of the block-hybrid sweep that must not change a bit: the speculative Gibbs step beside the
PS branch (option elb_spec, the default at small B) against PS first, then Gibbs; the ELB wavefront over two
CUs per chain (elb_parts) against one; the PHI block on the auxiliary
stream beside the ELB step (the default) against plain stream order (option phi_overlap = 0) -- the two
blocks touch disjoint state -- and the lag-structured CTA solve on two workgroups per chain (the
default at small B) against one (option solve_split = 0), and the forecast paths with the coefficients in
registers (the default for N <= 21) against PAI staged in LDS (option fcst_reg = 0) -- every sum in the
same order.  Every draw, the shadow rates, the forecasts and the status words are identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("var,B", [("phi_overlap", 8), ("solve_split", 8), ("solve_split", 1),
                                   ("fcst_reg", 8), ("elb_spec", 8), ("elb_spec", 1), ("elb_parts", 8),
                                   ("fcst_overlap", 8), ("fcst_overlap", 1)])
def test_schedule_bit_identical(pkg, ctx, fred, var, B):
    d = fred
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    bm = pkg.model.build_bh(len(d["ydates"]) - 1, p, 12, d["data"], d["ydates"], ndxS, ndxO, mpm, 0.25, e0, True)
    m = bm.var
    yields = np.zeros(m.N, bool)
    yields[ndxY] = True
    yreal = pkg.samplers.realized_values(d["data"], len(d["ydates"]) - 1, 12, ndxS, 0.25)
    nsw = 4
    outs = []
    for ov in (0, 1):
        ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, store_capacity=nsw, seed=77,
                        model=pkg.MODEL_BLOCKHYBRID, Ns=len(bm.ndxS), elbTmax=bm.elbT, elb_gibbsburn=20, elb=0.25,
                        options={var: ov})
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        ch.set_elb_model(bm.ndxS, bm.actual_block)
        ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
        ch.set_fcst(12, 4, yields, keep_paths=False)
        ch.set_fcst_slot(0, yreal[:, 0])
        ch.set_elb_ps(200, 3)
        st = pkg.model.initial_state(m, B)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        ch.sweep(nsw, store=True)
        outs.append((ch.get_state(), ch.get_shadowrate(), ch.get_fcst(), ch.get_draws(), ch.get_status()))
        ch.close()
    (s0, sh0, f0, d0, st0), (s1, sh1, f1, d1, st1) = outs
    for k in ("PAI", "A", "invA", "sqrtht", "h", "sqrtPHI", "PHI"):
        np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
    np.testing.assert_array_equal(sh0, sh1)
    for k in ("scores", "fYsum", "fYcsum"):
        np.testing.assert_array_equal(f0[k], f1[k], err_msg=k)
    for k in d0:
        np.testing.assert_array_equal(d0[k], d1[k], err_msg=k)
    np.testing.assert_array_equal(st0, st1)
