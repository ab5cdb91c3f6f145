"""The lag-structured CTA path (ccmm_lag.hip: D slab in LDS, intercept peeled,
explicit inverse factor as CTA.m:77) against the generic-X path (ccmm_gram_chol.hip +
ccmm_cta_solve.hip) and against the oracle, on the same common random numbers.

The generic path is selected with the chain set's option lag = 0."""

import numpy as np
import pytest

from conftest import rel_err
from helpers import crn_flat, random_state, toy_setup

pytestmark = pytest.mark.gpu


def _run_linear(pkg, ctx, oracle, su, m, B, nsweeps, no_lag, seed=21):
    sts = [random_state(oracle, su, seed=100 + c) for c in range(B)]
    rng = np.random.default_rng(seed)
    crns = [[oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI) for _ in range(nsweeps)]
            for _ in range(B)]
    ch = pkg.Chains(ctx, N=su.N, p=su.p, T=su.T, B=B, crn=True, options={"lag": 0 if no_lag else 1})
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_state(*[np.stack([s[k] for s in sts], -1) for k in ("PAI", "A", "sqrtht", "h",
                                                               "sqrtPHI")])
    flat = np.stack([np.stack([crn_flat(oracle, crns[c][m_], su) for m_ in range(nsweeps)], -1)
                     for c in range(B)], -1)
    ch.profile(True)
    ch.sweep(nsweeps, crn=flat)
    kt = ch.kernel_times()
    assert (kt["k_gram_chol_lag"][1] > 0) == (not no_lag), kt  # the path under test ran
    return ch.get_state(), sts, crns


@pytest.mark.parametrize("shape", ["toy", "real"])
def test_lag_vs_generic_path(pkg, ctx, oracle, fred, shape):
    """One CRN sweep: the two device paths agree to 5e-9 of max(|x|, posterior sd) and
    both sit at the oracle within the sweep tolerance of test_linear_sweep_crn."""
    if shape == "toy":
        su = toy_setup(oracle, N=4, p=2, Tobs=62, seed=5)
        data = np.vstack([su.X[0, 1:].reshape(su.p, su.N)[::-1], su.Y])
        m = pkg.model.build_var(data.shape[0], su.p, 12, data, np.arange(data.shape[0], dtype=float),
                                np.ones(su.N), True)
    else:
        mpm = oracle.set_minnesota_mean(fred["ncode"])
        su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
        m = pkg.model.build_var(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    np.testing.assert_array_equal(m.X, su.X)
    B = 3
    g_lag, sts, crns = _run_linear(pkg, ctx, oracle, su, m, B, 1, no_lag=False)
    g_gen, _, _ = _run_linear(pkg, ctx, oracle, su, m, B, 1, no_lag=True)
    for c in range(B):
        want = oracle.linear_sweep(sts[c], su, crns[c][0])
        _, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, want["A"], sts[c]["sqrtht"], su.iVdiag,
                              su.iVb, want["PAI"], np.zeros((su.K, su.N)), return_sd=True)
        d_paths = rel_err(g_lag["PAI"][..., c], g_gen["PAI"][..., c], sd)
        d_lag = rel_err(g_lag["PAI"][..., c], want["PAI"], sd)
        d_gen = rel_err(g_gen["PAI"][..., c], want["PAI"], sd)
        print(shape, c, "lag-generic", d_paths, "lag-oracle", d_lag, "generic-oracle", d_gen)
        assert d_paths < 5e-8 and d_lag < 5e-8, (d_paths, d_lag, d_gen)
        assert rel_err(g_lag["sqrtht"][..., c], want["sqrtht"]) < 5e-8
