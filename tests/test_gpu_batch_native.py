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
        "PAIstdev", "countELBaccept", "shadowrateVintagesMid", "shadowrateVintagesTails")
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
