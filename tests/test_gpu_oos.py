"""GPU tests of the block-hybrid quasi-real-time OOS batch
(samplers.goVARshadowrateBlockHybrid_batch; goVARshadowrateBlockHybrid.m:126-517): every
vintage is a data slot of one device-resident chain set, kept sweeps forecast on the
device, log scores are reduced per vintage (log mean exp, :437-447).

  * all 164 real-data vintages (jump-offs after 2008-12, T = 587..750, elbT = 2..165) run
    a few sweeps in one chain set;
  * two ranks (gloo, both on cuda:0) shard the vintages longest-processing-time first and
    all-gather the summaries: every rank's table equals the one-rank run (Philox streams
    keyed by the global unit, so sharding does not change the draws)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _setup(pkg, fred):
    ndxS, ndxO, _ = pkg.model.setShadowYields(fred["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(fred["ncode"])
    return ndxS, ndxO, mpm


def test_bh_batch_all_vintages(pkg, fred):
    ndxS, ndxO, mpm = _setup(pkg, fred)
    out = pkg.samplers.goVARshadowrateBlockHybrid_batch(
        fred["data"], fred["ydates"], ndxS, ndxO, mpm, MCMCdraws=2, burnin=2, fcstNdraws=4,
        fcstNhorizons=12, gibbsburn=5, nchains=1)
    T = out["Tjumpoffs"]
    assert len(T) == 164 and T[0] == 599 and T[-1] == 762          # 2009-01 .. 2022-08 (1-based)
    assert out["stats"]["retries"] == []
    ls = out["fcstYmvlogscore"]
    # the last vintage has no realized data: NaN scores; every other vintage is finite
    assert np.all(np.isfinite(ls[:-1])) and np.isnan(ls[-1])
    assert np.all(np.isfinite(out["fcstYmvlogscoreX"][:-1]))
    assert np.all(np.isfinite(out["fcstYhat"])) and out["fcstYhat"].shape == (20, 12, 164)
    # censored forecasts of the yields sit at or above the ELB; shadow forecasts need not
    yi = np.union1d(ndxS, ndxO)
    assert np.all(out["fcstYhat"][yi] >= 0.25 - 1e-12)
    # shadow-rate medians exist on the vintage's ELB window only
    mid = out["shadowrateVintagesMid"]
    for v in (0, 80, 163):
        thisT = T[v]
        w = mid[:, :, v]
        assert np.all(np.isfinite(w[597:thisT])) and np.all(np.isnan(w[:597]))
        assert np.all(np.isnan(w[thisT:]))
    st = out["stats"]
    assert st["units_local"] == 164 and st["sweeps_local"] == 164 * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


KW = dict(MCMCdraws=3, burnin=2, fcstNdraws=6, fcstNhorizons=6, gibbsburn=4, nchains=2,
          Tjumpoffs=[600, 640, 700, 740, 761])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    from oracle import ccmm_oracle as O  # CSV loader only
    fred = O.load_fred_csv(Path(__file__).resolve().parent / "golden/data/fredblockMD20-2022-09.csv")
    dist, w = pkg.distributed.init("gloo")
    ndxS, ndxO, mpm = _setup(pkg, fred)
    out = pkg.samplers.goVARshadowrateBlockHybrid_batch(fred["data"], fred["ydates"], ndxS, ndxO,
                                                        mpm, dist=dist, device=0, **KW)
    q.put((w.rank, {k: out[k] for k in ("fcstYmvlogscore", "fcstYmvlogscoreX", "fcstYhat",
                                         "PAImean", "shadowrateVintagesMid")},
           out["assignment"], out["stats"]["vintages_local"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bh_batch_gloo_world2_matches_world1(pkg, fred):
    ndxS, ndxO, mpm = _setup(pkg, fred)
    ref = pkg.samplers.goVARshadowrateBlockHybrid_batch(fred["data"], fred["ydates"], ndxS, ndxO,
                                                        mpm, **KW)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=280) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    nloc = 0
    for rank, got, assign, nv in res:
        nloc += nv
        assert sorted(assign[0] + assign[1]) == list(range(5)) and assign[0] and assign[1]
        for k, v in got.items():
            a, b = np.asarray(v), np.asarray(ref[k])
            fin = np.isfinite(b)
            assert np.array_equal(np.isfinite(a), fin), k
            err = np.max(np.abs(a[fin] - b[fin]) / np.maximum(np.abs(b[fin]), 1.0))
            assert err < 1e-8, (k, err)
    assert nloc == 5
