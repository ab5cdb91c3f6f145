"""Five shadow rates (setShadowYields.m:1-5: the Krippner / Wu-Xia datasets at ELB > 0.25 add
KRIPPNERSHADOWRATE or WUXIASHADOWRATE and GS5 to FEDFUNDS, TB3MS / TB6MS, GS1): the block-hybrid
sweep (ELB Gibbs step with Ns = 5 conditionals, k_elb_cond<5> / k_elb_gibbs_wf<5, 8>) and the PS
branch with a censored-cell band width above 64 (Ns (p + 1) = 65 at p = 12: the 80-wide proposal
kernels), both against the oracle under common random numbers."""
import numpy as np
import pytest

from helpers import synth_bh_data, toy_bh_setup
from test_gpu_bh import _check as bh_check
from test_gpu_bh import _run as bh_run
from test_gpu_ps import _check as ps_check
from test_gpu_ps import _run as ps_run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bh():
    from oracle import ccmm_oracle_bh
    return ccmm_oracle_bh


def test_bh_sweep_crn_ns5(pkg, ctx, oracle, bh):
    """N = 7, p = 2, five shadow rates (the odd ones with uncensored months in the window), one
    other yield: two CRN sweeps, draws, KSC indicators and truncated-normal branches."""
    bs = toy_bh_setup(bh, N=7, p=2, ndxS=(1, 2, 3, 4, 5), ndxO=(6,), seed=11)
    assert len(bs.ndxS) == 5
    out = bh_run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=2, seed=70)
    bh_check(oracle, bs, *out, tol_pai=1e-9, tol_s=1e-9)


def test_ps_ns5_band_width_above_64(pkg, ctx, oracle, bh):
    """N = 6, p = 12, five shadow rates censored together over 40 months: the censored-cell
    precision has band width 5 (12 + 1) = 65, past the 64-wide proposal kernels."""
    N, p, Tobs, ndxS, ndxO = 6, 12, 170, (0, 1, 2, 3, 4), (5,)
    data = synth_bh_data(N, p, Tobs, elb_window=(120, 160), ndxS=ndxS, seed=5)
    rng = np.random.default_rng(6)
    for s in ndxS:                                  # every rate censored in every window month
        data[120:160, s] = 0.25 - rng.uniform(0.01, 0.2, 40)
    hit = np.any(data[:, list(ndxS)] <= 0.25, axis=1)
    bs = bh.bh_setup(Tobs, p, 12, data, np.arange(Tobs, dtype=float), np.asarray(ndxS), np.asarray(ndxO),
                     np.ones(N), 0.25, int(np.argmax(hit)) - p)
    assert len(bs.ndxS) == 5 and bs.sNaN[:, :40].all()   # band width 5 (p + 1) = 65
    got, S, ps, want = ps_run(pkg, ctx, oracle, bh, bs, B=2, nsweeps=2, NP=64, seed=13)
    ps_check(oracle, bs, got, S, ps, want, 1e-9)
