"""GPU parity of the predictive-density block (ccmm_fcst, k_fcst) against
oracle/ccmm_oracle_fcst.fcst_draw (mcmcVAR.m:298-381, logscoreGaussian.m,
logscoreGaussianCensored.m) with common random numbers, on a real-data kept draw
(N=20, p=12, K=241, H=48, Nd=10, 4 chains).

Tolerances: simulated paths 1e-9 in |Δ| / max(|x|, 1) (48-step recursions in a
different summation order); log scores 1e-9 absolute + relative for one and two
censored series (normcdf / Genz BVN against the oracle's adaptive quadrature),
1e-8 for three (graded Gauss-Legendre outer integral on the device; MATLAB's own
trivariate mvncdf tolerance is 1e-8 absolute).  Four or more censored series: MATLAB
mvncdf is randomised quasi-Monte Carlo (tolerance 1e-4); device and oracle evaluate the declared
deterministic lattice rule (oracle.mvn_lattice_cdf, itself within 1e-6 of scipy's Genz lattice in
tests/test_oracle_fcst.py) and agree to 1e-8 (the conditional factor of Omega and the deep-tail
inverse CDFs differ in the last bits; measured 1.4e-9 at four series)."""
import numpy as np
import pytest

from conftest import rel_err
from fcst_cases import fcst_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    from oracle import ccmm_oracle_fcst
    return ccmm_oracle_fcst


def _oracle(F, d, y, B):
    outs = [F.fcst_draw(d["PAI"][..., c], d["invA"][..., c], d["logSV0"][:, c], d["sqrtPHI"][..., c],
                        d["Xj"][:, c], y, d["yields"], d["elb"], d["svz"][..., c], d["z"][..., c])
            for c in range(B)]
    return [np.stack([o[k] for o in outs], axis=-1) for k in range(4)]


@pytest.mark.parametrize("case", [0, 1, 2, 3])
def test_fcst_crn(ctx, oracle, fred, F, case):
    B = 4
    d = fcst_inputs(oracle, fred, B=B)
    y = d["ys"][case]
    fY, fYc, yhat, sc, st = ctx.fcst(d["PAI"], d["invA"], d["logSV0"], d["sqrtPHI"], d["Xj"], y,
                                     d["yields"], d["elb"], d["H"], d["Nd"], d["svz"], d["z"])
    rfY, rfYc, ryhat, rsc = _oracle(F, d, y, B)
    assert np.all(st == 0)
    e = rel_err(yhat, ryhat, 1.0)
    assert e < 1e-9, e
    assert rel_err(fY, rfY, 1.0) < 1e-9
    assert rel_err(fYc, rfYc, 1.0) < 1e-9
    assert np.array_equal(fYc[d["yields"]] == d["elb"], rfYc[d["yields"]] == d["elb"])  # censoring flags
    e = rel_err(sc, rsc, 1.0)
    assert e < (1e-8 if case == 3 else 1e-9), e


@pytest.mark.parametrize("nat", [4, 6])
def test_fcst_four_or_more_at_elb(ctx, oracle, fred, F, nat):
    """4 and 6 yields at the ELB: the censored scores (fcstLogscoreDraws, fcstLogscoreIdraws) go
    through the lattice mvncdf rule on the device and in the oracle."""
    B = 2
    d = fcst_inputs(oracle, fred, B=B, nat=(nat,))
    y = d["ys"][0]
    fY, fYc, yhat, sc, st = ctx.fcst(d["PAI"], d["invA"], d["logSV0"], d["sqrtPHI"], d["Xj"], y,
                                     d["yields"], d["elb"], d["H"], d["Nd"], d["svz"], d["z"])
    assert np.all(st == 0) and not np.any(np.isnan(sc))
    rfY, rfYc, ryhat, rsc = _oracle(F, d, y, B)
    assert rel_err(fY, rfY, 1.0) < 1e-9 and rel_err(fYc, rfYc, 1.0) < 1e-9
    # probabilities that underflow give log(0) = -Inf on both sides (MATLAB's log as well)
    np.testing.assert_array_equal(np.isinf(sc), np.isinf(rsc))
    fin = np.isfinite(rsc)
    e = rel_err(sc[fin], rsc[fin], 1.0)
    print(f"{nat} at the ELB: censored scores {sc[1, :3, 0]} vs {rsc[1, :3, 0]}, max err {e:.1e}")
    assert e < 1e-8, e


def test_fcst_philox(ctx, oracle, fred, F):
    """Generated draws: RNG-free outputs (mean path, censoring floor) and moment checks."""
    B = 64
    d = fcst_inputs(oracle, fred, B=4)
    rep = lambda a: np.repeat(a[..., :1], B, axis=-1)
    y = d["ys"][0]
    fY, fYc, yhat, sc, st = ctx.fcst(rep(d["PAI"]), rep(d["invA"]), rep(d["logSV0"]),
                                     rep(d["sqrtPHI"]), rep(d["Xj"]), y, d["yields"], d["elb"],
                                     d["H"], d["Nd"], seed=1012023, sweep=3)
    _, _, ryhat, _ = F.fcst_draw(d["PAI"][..., 0], d["invA"][..., 0], d["logSV0"][:, 0],
                                 d["sqrtPHI"][..., 0], d["Xj"][:, 0], y, d["yields"], d["elb"],
                                 d["svz"][..., 0], d["z"][..., 0])
    e = rel_err(yhat, ryhat[..., None], 1.0)
    assert e < 1e-9, e
    assert np.all(fYc[d["yields"]] >= d["elb"]) and np.all(np.isfinite(sc))
    # one-step draws: mean = yhat(:,1), covariance invA diag(exp(logSV0)) invA' up to SV noise
    e1 = fY[:, 0, :, :].reshape(fY.shape[0], -1) - yhat[:, 0, :1]
    sd = np.sqrt(np.diag(d["invA"][..., 0] @ np.diag(np.exp(d["logSV0"][:, 0])) @ d["invA"][..., 0].T))
    z = e1.mean(axis=1) / (sd / np.sqrt(e1.shape[1]))
    assert np.max(np.abs(z)) < 5.0
    ratio = e1.std(axis=1) / sd
    assert np.all((ratio > 0.85) & (ratio < 1.2))
    # draws differ across chains (chain index is part of the Philox counter)
    assert not np.allclose(fY[..., 0], fY[..., 1])


def test_mcmcVAR_predictive_density(pkg, oracle, fred, F):
    """samplers.mcmcVAR with fcstNdraws (nargout 15): kept-draw loop + ccmm_fcst.
    RNG-free end-to-end check: fcstYhatRB = mean over kept draws of the zero-shock
    path of each stored PAI draw (mcmcVAR.m:375-379, :400)."""
    sel = [0, 4, 14, 17]  # two macro series, FEDFUNDS-like and a yield (ndxYIELDS = [2, 3])
    data = fred["data"][-120:, sel]
    ydates = fred["ydates"][-120:]
    mpm = np.ones(len(sel))
    T0 = len(ydates) - 6
    yreal = data[T0:T0 + 6].T
    M, Nd_total, H = 20, 40, 6
    out = pkg.samplers.mcmcVAR(T0, M, 2, 12, data, ydates, mpm, True, ndxYIELDS=[2, 3],
                               ELBbound=0.25, yrealized=yreal, fcstNdraws=Nd_total,
                               fcstNhorizons=H, rndStream=7, burnin=10)
    assert len(out) == 15
    PAI_all, fYd, fYhat, fYcd, yhatRB, ls = out[0], out[4], out[5], out[6], out[10], out[11]
    assert fYd.shape == (4, H, Nd_total) and fYcd.shape == (4, H, Nd_total) and ls.shape == (Nd_total,)
    assert np.all(fYcd[[2, 3]] >= 0.25) and np.all(np.isfinite(ls))
    assert np.allclose(fYhat, fYd.mean(axis=2))
    m = pkg.model.build_var(T0, 2, 12, data, ydates, mpm, True)
    want = np.zeros((4, H))
    for d in range(M):
        P = PAI_all[d]
        x = m.Xjumpoff.copy()
        for hh in range(H):
            yv = P.T @ x
            x = np.concatenate([[1.0], yv, x[1:1 + 4 * (2 - 1)]])
            want[:, hh] += yv / M
    e = rel_err(yhatRB, want, 1.0)
    assert e < 1e-8, e


def test_goVAR_batch_gpu(pkg, fred):
    """goVAR_batch (world 1) over two real-data vintages with mcmcVAR + ccmm_fcst:
    per-vintage log mean exp of the returned log-score draws, fcstYhat per vintage."""
    sel = [0, 4, 14, 17]
    data = fred["data"][-140:, sel]
    ydates = fred["ydates"][-140:]
    res = pkg.samplers.goVAR_batch(data, ydates, [120, 128], 2, 12, 10, 20, 4, np.ones(4), [2, 3],
                                   nchains=2, burnin=5)
    assert res["fcstYmvlogscore"].shape == (2,) and np.all(np.isfinite(res["fcstYmvlogscore"]))
    assert res["fcstYhat"].shape == (4, 4, 2) and np.all(np.isfinite(res["fcstYhat"]))
    assert np.all(res["fcstYmvlogscoreX"] > -1e3) and np.all(res["fcstYmvlogscoreI"] > -1e3)
