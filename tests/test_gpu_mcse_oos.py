"""Posterior-level check of one quasi-real-time OOS vintage (goVARshadowrateBlockHybrid.m:258-456):
the vintage's predictive density from 128 Philox device chains against long oracle chains
(tests/golden/mcse_oos_vintage.npz, tools/make_mcse_oos_fixture.py: seven pooled chains of 1000 burn-in
+ 2000 kept sweeps with the reference's ELB schedule, 10 forecast paths x 48 horizons per kept sweep).

Quantities (per kept sweep, averaged over the window): the one-step predictive density at the
realised values (dens: mean of exp(fcstLogscoreDraws); fcstYmvlogscore = log of its posterior mean,
:437-439), the mean log score, and the mean censored path fcstYhat (:450) of every variable at
horizons 1, 12, 24 and 48.  Each within 4.5 combined standard errors (oracle: the larger of the pooled
NSE and the spread of the seven chain means; device: the spread of the 128 chain means / sqrt(128)).
The device run follows the batch driver's chain set (samplers._bh_chain_set: the vintage's data slot,
reference initialisation, per-chain Philox streams, PS proposals from m >= MCMCburnin / 2)."""
import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_oos_vintage_predictive_density_within_mcse(pkg, ctx, fred):
    path = ROOT / "tests" / "golden" / "mcse_oos_vintage.npz"
    if not path.exists():
        pytest.fail(f"{path.name} missing: run tools/make_mcse_oos_fixture.py")
    g = np.load(path)
    S = pkg.samplers
    d = fred
    ELB, H, Nd = 0.25, 48, 10
    thisT = int(g["thisT"])
    hsel = [int(h) for h in g["hsel"]]
    burn, keep = int(g["burn"]), int(g["keep"])
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], ELB)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    e0 = pkg.model.elbT0_of(d["data"], ndxS, ELB, 12)
    units = S._bh_units(d["data"], d["ydates"], [thisT], 12, 12, ndxS, ndxO, mpm, ELB, e0, True, H)
    B, chunk = 128, 50
    ch, _, _ = S._bh_chain_set(ctx, units, B, seed=4242, ids=np.arange(B, dtype=np.uint32), store_capacity=chunk,
                               gibbsburn=100, ELBbound=ELB, ndxYIELDS=ndxY, fcstNhorizons=H, Nd=Nd)
    ch.set_elb_ps(int(g["nproposals"]), -(-burn // 2))       # m >= MCMCburnin / 2 (:435)
    for done in range(0, burn, chunk):
        ch.sweep(min(chunk, burn - done), store=False)
    N = units[0][1].var.N
    dens = np.zeros(B)
    lsc = np.zeros(B)
    paths = np.zeros((N, len(hsel), B))
    for done in range(0, keep, chunk):
        n = min(chunk, keep - done)
        ch.sweep(n, store=True)
        fc = ch.get_fcst()
        ch.get_draws()                                          # drains the draw store for the next chunk
        sc = fc["scores"][:, :, 1, :]                           # Nd x n x B: fcstLogscoreDraws
        dens += np.exp(sc).mean(axis=0).sum(axis=0)
        lsc += sc.mean(axis=0).sum(axis=0)
        paths += fc["fYcsum"][:, hsel, :] / Nd                   # censored paths summed over draws
    status = ch.get_status()
    ch.close()
    assert not np.any(status & ~65), status
    means = np.vstack([dens / keep, lsc / keep, (paths / keep).reshape(N * len(hsel), B, order="F")])
    m_gpu = means.mean(axis=1)
    nse_gpu = means.std(axis=1, ddof=1) / np.sqrt(B)
    se_o = np.maximum(g["nse3"], g["se_between"])
    z = (m_gpu - g["pmean"]) / np.sqrt(se_o ** 2 + nse_gpu ** 2)
    print(f"vintage thisT {thisT}: {z.size} quantities, max |z| {np.abs(z).max():.2f}, median {np.median(np.abs(z)):.2f}")
    print(f"  fcstYmvlogscore: device {np.log(m_gpu[0]):.4f}, oracle {np.log(g['pmean'][0]):.4f} "
          f"(relative SEs {nse_gpu[0] / m_gpu[0]:.3f} / {se_o[0] / g['pmean'][0]:.3f}); "
          f"mean log score {m_gpu[1]:.4f} vs {g['pmean'][1]:.4f}")
    for q in np.argsort(-np.abs(z))[:4]:
        print(f"  q{q}: gpu {m_gpu[q]:.5g} +- {nse_gpu[q]:.3g}  oracle {g['pmean'][q]:.5g} +- {se_o[q]:.3g}  z {z[q]:.2f}")
    assert np.abs(z).max() < 4.5, np.round(z, 2)
