"""The C-level vintage loop ccmm_run_batch (include/ccmm.h; the parfor over vintages of
goVARshadowrateBlockHybrid.m:258-517 / goVARhybrid.m:258 as one device-resident chain set with
burn-in, kept sweeps, forecast records, device summaries and retries inside the library)
against the Python driver over the same chain-set API (samplers.goVARshadowrateBlockHybrid_batch,
engine="python"): the same Philox streams (unit = vintage index x nchains + chain) give the same
draws, so every per-vintage output agrees to host summation order (1e-12)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("fcstYmvlogscore", "fcstYmvlogscoreX", "fcstYmvlogscoreI", "fcstYhat", "fcstShadowYhat", "PAImean",
        "PAIstdev", "countELBaccept", "shadowrateVintagesMid", "shadowrateVintagesTails", "shadowratePSRF")
POST = ("fcstYmedian", "fcstYcrps", "fcstYquantiles", "fcstYcummedian", "fcstYcumcrps", "fcstYcumquantiles",
        "fcstShadowYmedian", "fcstShadowYquantiles", "PAImedian", "PAIquantiles", "fcstYmvlogscoreDraws",
        "fcstYmvlogscoreXdraws", "fcstYmvlogscoreIdraws", "fcstYcumhat", "fcstYcumrealized")


def _cmp(a, b, keys):
    for k in keys:
        x, y = np.asarray(a[k], float), np.asarray(b[k], float)
        assert x.shape == y.shape, (k, x.shape, y.shape)
        assert np.array_equal(np.isnan(x), np.isnan(y)), k
        m = ~np.isnan(x)
        err = float(np.max(np.abs(x[m] - y[m]) / np.maximum(np.abs(y[m]), 1.0))) if m.any() else 0.0
        print(f"  {k}: max rel {err:.2e}")
        assert err < 1e-12, (k, err)


@pytest.mark.parametrize("model,postprocess", [("blockhybrid", False), ("blockhybrid", True), ("hybrid", True)])
def test_native_batch_matches_python_driver(pkg, fred, model, postprocess):
    S = pkg.samplers
    d = fred
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    nT = len(d["ydates"])
    Tj = [nT - 150, nT - 60, nT - 12, nT]                 # the last vintage has no realized data
    kw = dict(Tjumpoffs=Tj, MCMCdraws=8, fcstNdraws=16, burnin=8, gibbsburn=5, nchains=2, chunk=3,
              postprocess=postprocess, cumcode=d["cumcode"] if postprocess else None, Nproposals=64,
              model=model, fcstNhorizons=24)
    ref = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, engine="python", **kw)
    nat = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, engine="native", **kw)
    print(model, "postprocess", postprocess, "accepts", nat["countELBaccept"])
    _cmp(nat, ref, KEYS + (POST if postprocess else ()))
    assert np.all(np.isfinite(nat["fcstYmvlogscore"][:-1])) and np.isnan(nat["fcstYmvlogscore"][-1])


def test_native_batch_argument_errors(pkg, ctx):
    with pytest.raises(RuntimeError, match="fcstNdraws must be multiple"):
        ctx.run_batch(model=pkg.MODEL_BLOCKHYBRID, N=4, p=2, Ns=1, ndxS=[0], actual_block=np.ones(4, bool),
                      ndxYields=np.zeros(4, bool), nchains=1, MCMCdraws=4, burnin=0, gibbsburn=1, Nproposals=0,
                      fcstNdraws=6, H=2, elb=0.25, seed=1, chunk=2, max_retries=0, postprocess=False, pct=(),
                      cumcode=None, vintages=[])
    with pytest.raises(RuntimeError, match="ndxYields required"):       # NULL ndxYields: an error, not a crash
        ctx.run_batch(model=pkg.MODEL_BLOCKHYBRID, N=4, p=2, Ns=1, ndxS=[0], actual_block=np.ones(4, bool),
                      ndxYields=None, nchains=1, MCMCdraws=4, burnin=0, gibbsburn=1, Nproposals=0,
                      fcstNdraws=4, H=2, elb=0.25, seed=1, chunk=2, max_retries=0, postprocess=False, pct=(),
                      cumcode=None, vintages=[])


@pytest.mark.parametrize("model,C", [("blockhybrid", 1), ("blockhybrid", 3), ("hybrid", 1)])
def test_shadowrate_psrf_matches_oracle(pkg, fred, model, C):
    """shadowratePSRF (goVARshadowrateBlockHybrid.m:322-325 / goVARhybrid.m:322-323): per vintage and
    shadow rate, DiagnosticsShadowrate = mean of psrf (DiagnosticsShadowrate.m:34-128) over the kept
    draws of the months at the ELB, ELBdummy(startELB:thisT, s).  Checked against the oracle's psrf
    on the kept draws the run returns (1e-12), on both engines."""
    from oracle.ccmm_oracle_stats import diagnostics_shadowrate, diagnostics_shadowrate_chain_mean
    S = pkg.samplers
    d = fred
    ELB = 0.25
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], ELB)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    nT = len(d["ydates"])
    Tj = [nT - 160, nT - 100, nT - 30, nT]
    kw = dict(Tjumpoffs=Tj, MCMCdraws=30, fcstNdraws=30, burnin=6, gibbsburn=5, nchains=C, chunk=10,
              Nproposals=64, model=model, fcstNhorizons=6)
    ref = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, keep_draws=True, **kw)
    nat = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, engine="native", **kw)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, ELB, 12)
    startELB = e0 + 1 + 12
    dummy = d["data"][:, ndxS] <= ELB                                  # ELBdummy (:131)
    assert ref["shadowratePSRF"].shape == (len(ndxS), len(Tj))
    worst = 0.0
    for v, thisT in enumerate(Tj):
        sr = ref["shadowrate_all"][v]                                  # M x Ns x elbT x C
        mask = dummy[startELB - 1:thisT]                               # elbT x Ns
        assert sr.shape[2] == mask.shape[0]
        for s in range(len(ndxS)):
            cells = sr[:, s][:, mask[:, s], :]                         # M x nObs x C
            want = diagnostics_shadowrate_chain_mean(cells)          # the reference's one-chain statistic
            wantc = diagnostics_shadowrate(cells) if C > 1 else np.nan  # psrf across the chains
            for key, w in (("shadowratePSRF", want), ("shadowratePSRFchains", wantc)):
                for got in (ref[key][s, v], nat[key][s, v]):
                    if np.isnan(w):
                        assert np.isnan(got), (key, v, s)
                        continue
                    err = abs(got - w) / max(1.0, abs(w))
                    worst = max(worst, err)
                    assert err < 1e-12, (key, v, s, got, w)
    print(f"  {model} C={C}: shadowratePSRF {ref['shadowratePSRF'].round(3).tolist()} max rel {worst:.2e}")
    assert np.all(np.isfinite(ref["shadowratePSRF"][:, 1:]))
