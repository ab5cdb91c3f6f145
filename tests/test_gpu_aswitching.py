"""GPU parity of the CTAsysAswitching drop-in (CTAsysAswitching.m:1-123, the coefficient block
of the Aelb shadow-rate model): the months at the ELB use a second A matrix Aelb_ in the
residual map and the kron weights (:61-80).  On the device this is the weighted SYRK with a
per-month choice of A in the weights and in v_t (ccmm_cta_aswitching).

Against the oracle as written (oracle.cta_sys_aswitching: the kron-materialised at-ELB rows
stacked over the away rows, explicit inverse), Cholesky branch and the QR branch of :82-93
(CCMM_FORCE_QR=1: host Householder QR of Kailath's array with the same two-matrix map).
Tolerance: |delta| / max(|x|, sd_post) < 1e-9."""

import numpy as np
import pytest

from conftest import rel_err
from helpers import random_state, toy_setup

pytestmark = pytest.mark.gpu


def _case(oracle, seed=2):
    su = toy_setup(oracle, N=5, p=3, Tobs=90, seed=seed)
    rng = np.random.default_rng(9)
    XX = np.repeat(su.X[:, :, None], su.N, axis=2)
    XX[:, 1:, 3:] += 0.1 * rng.standard_normal((su.T, su.K - 1, su.N - 3))   # two design slabs
    at = np.zeros(su.T, bool)
    at[30:61] = True                                                         # an ELB episode
    at[70:74] = True
    sts = [random_state(oracle, su, seed=8 + c) for c in range(2)]
    Aelb = [np.eye(su.N) + np.tril(rng.uniform(-0.4, 0.4, (su.N, su.N)), -1) for _ in sts]
    zs = [rng.standard_normal((su.K, su.N)) for _ in sts]
    return su, XX, at, sts, Aelb, zs


def _check(ctx, oracle, force):
    su, XX, at, sts, Aelb, zs = _case(oracle)
    got, status = ctx.cta_aswitching(su.Y, XX, np.stack([s["A"] for s in sts], -1), np.stack(Aelb, -1), at,
                                     np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb,
                                     np.stack([s["PAI"] for s in sts], -1), np.stack(zs, -1))
    assert np.all(status == (1 if force else 0))
    for c in range(len(sts)):
        want, st, sd = oracle.cta_sys_aswitching(su.Y, XX, su.N, su.K, su.T, sts[c]["A"], Aelb[c], at,
                                                 sts[c]["sqrtht"], su.iVdiag, su.iVb, sts[c]["PAI"], zs[c],
                                                 return_sd=True, force_qr=force)
        e = rel_err(got[..., c], want, sd)
        # the switch matters: the single-A draw is far from the two-matrix one
        plain, _, _ = oracle.cta_sys(su.Y, XX, su.N, su.K, su.T, sts[c]["A"], sts[c]["sqrtht"], su.iVdiag,
                                     su.iVb, sts[c]["PAI"], zs[c], return_sd=True)
        print("aswitching", "qr" if force else "chol", "chain", c, e, "vs single-A", rel_err(plain, want, sd))
        assert e < 1e-9, e
        assert rel_err(plain, want, sd) > 1e-3


def test_cta_aswitching(ctx, oracle):
    _check(ctx, oracle, False)


def test_cta_aswitching_qr_branch(ctx, oracle):
    with ctx.options(force_qr=1):
        _check(ctx, oracle, True)


def test_cta_aswitching_all_away_equals_ctasys(ctx, oracle):
    """atELB all false: the drop-in reduces to CTAsys (same device path, bit for bit)."""
    su, XX, at, sts, Aelb, zs = _case(oracle, seed=4)
    at[:] = False
    args = (np.stack([s["A"] for s in sts], -1),)
    rest = (np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb, np.stack([s["PAI"] for s in sts], -1),
            np.stack(zs, -1))
    g1, _ = ctx.cta_aswitching(su.Y, XX, args[0], np.stack(Aelb, -1), at, *rest)
    g0, _ = ctx.cta(su.Y, XX, args[0], *rest)
    np.testing.assert_array_equal(g1, g0)
