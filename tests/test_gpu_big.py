"""GPU parity of the large-system coefficient block (ccmm_big.hip: multi-equation FP64-MFMA
Gram, per-system blocked Cholesky, per-chain sequential solve; CTA.m:57-98 /
CTAsys.m:57-108) against the oracle (as written: kron-materialised X_j, explicit inverse).

The large path serves K > 512 or N > 32 (the S120 configuration); option large_path = 1 routes
the N = 20 / K = 241 shapes through it too, so it is checked on the same cases as the
lag-structured path.  Tolerance: |Δ| / max(|x|, sd_post) as tests/test_gpu_parity.py."""

import numpy as np
import pytest

from conftest import rel_err
from helpers import random_state, toy_setup

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_big(ctx):
    with ctx.options(large_path=1):  # the block-level calls and the chain sets created in the test
        yield


def _cta(oracle, ctx, su, sts, rng, XX=None):
    B = len(sts)
    zs = [rng.standard_normal((su.K, su.N)) for _ in range(B)]
    P0 = [s["PAI"] + 0.01 * rng.standard_normal(s["PAI"].shape) for s in sts]
    X = su.X if XX is None else XX
    got, status = ctx.cta(su.Y, X, np.stack([s["A"] for s in sts], -1),
                          np.stack([s["sqrtht"] for s in sts], -1), su.iVdiag, su.iVb,
                          np.stack(P0, -1), np.stack(zs, -1))
    assert not status.any()
    errs = []
    for c in range(B):
        if XX is None:
            want, _, sd = oracle.cta(su.Y, su.X, su.N, su.K, sts[c]["A"], sts[c]["sqrtht"], su.iVdiag,
                                     su.iVb, P0[c], zs[c], return_sd=True)
        else:
            want, _, sd = oracle.cta_sys(su.Y, XX, su.N, su.K, su.T, sts[c]["A"], sts[c]["sqrtht"],
                                         su.iVdiag, su.iVb, P0[c], zs[c], return_sd=True)
        errs.append(rel_err(got[..., c], want, sd))
    return max(errs)


def test_big_cta_toy(ctx, oracle, force_big):
    su = toy_setup(oracle, N=4, p=2, Tobs=62)
    e = _cta(oracle, ctx, su, [random_state(oracle, su, seed=10 + c) for c in range(3)],
             np.random.default_rng(3))
    assert e < 1e-9, e


def test_big_cta_real_smooth(ctx, oracle, fred, force_big):
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    su = oracle.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
    e = _cta(oracle, ctx, su, [random_state(oracle, su, seed=5 + c) for c in range(2)],
             np.random.default_rng(4))
    print("big cta real smooth rel err (sd units)", e)
    # cond(iV_post) ~ 1e9 here: the large path's 64-row MFMA k-steps reorder the Gram sums
    # against the oracle's kron form; measured 1.05e-8 sd (the lag path: 4.5e-9)
    assert e < 3e-8, e


def test_big_ctasys_per_equation_designs(ctx, oracle, force_big):
    su = toy_setup(oracle, N=5, p=3, Tobs=90, seed=2)
    rng = np.random.default_rng(9)
    XX = np.repeat(su.X[:, :, None], su.N, axis=2)
    XX[:, 1:, 3:] += 0.1 * rng.standard_normal((su.T, su.K - 1, su.N - 3))  # two slabs
    e = _cta(oracle, ctx, su, [random_state(oracle, su, seed=8 + c) for c in range(2)], rng, XX)
    assert e < 1e-9, e


def test_big_cta_k1441(ctx, oracle):
    """K = 1441 regressors (the S120 design width; KP = 1472, 23 block columns), T = 750,
    six equations, a free-form design [1, Gaussian columns]: the large path without
    forcing."""
    rng = np.random.default_rng(21)
    T, N, K = 750, 6, 1441
    X = np.hstack([np.ones((T, 1)), rng.standard_normal((T, K - 1))])
    B0 = 0.02 * rng.standard_normal((K, N))
    A = np.eye(N) + np.tril(rng.uniform(-0.3, 0.3, (N, N)), -1)
    h = np.cumsum(0.05 * rng.standard_normal((T, N)), axis=0)
    E = rng.standard_normal((T, N)) * np.exp(h / 2)
    Y = X @ B0 + np.linalg.solve(A, E.T).T
    iVdiag = np.full((K, N), 4.0)
    iVb = np.zeros((K, N))
    sqrtht = np.exp(h / 2)
    P0 = B0 + 0.01 * rng.standard_normal((K, N))
    z = rng.standard_normal((K, N))
    got, status = ctx.cta(Y, X, A[..., None], sqrtht[..., None], iVdiag, iVb, P0[..., None],
                          z[..., None])
    assert not status.any()
    want, _, sd = oracle.cta(Y, X, N, K, A, sqrtht, iVdiag, iVb, P0, z, return_sd=True)
    e = rel_err(got[..., 0], want, sd)
    print("big cta K=1441 rel err (sd units)", e)
    assert e < 1e-9, e
