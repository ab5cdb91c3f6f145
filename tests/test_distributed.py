"""World-size-2 gloo tests (CPU) of the multi-GPU layer: sharding covers every
unit exactly once, LPT balances vintage costs, end-of-run reductions are exact."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_lpt_and_shards(pkg):
    dm = pkg.distributed
    costs = [dm.unit_cost(T, 241, 20, n_cens=max(0, T - 585) // 2) for T in range(587, 751)]
    for W in (1, 2, 4, 8):
        parts = dm.lpt_assign(costs, W)
        flat = sorted(u for p in parts for u in p)
        assert flat == list(range(len(costs)))
        loads = [sum(costs[u] for u in p) for p in parts]
        assert max(loads) / (sum(loads) / W) < 1.02
        spans = [dm.shard_range(256, W, r) for r in range(W)]
        assert spans[0][0] == 0 and spans[-1][1] == 256
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import __graft_entry__
    dm = __graft_entry__.load_package().distributed
    dist, w = dm.init("gloo")
    costs = np.arange(1, 11, dtype=float)
    mine = dm.lpt_assign(costs, w.size)[w.rank]
    local = {u: np.full(3, float(u)) for u in mine}
    allu = dm.gather_summaries(dist, local, None)
    tot = dm.allreduce_sum(dist, np.array([sum(costs[u] for u in mine), len(mine)]))
    rng = np.random.default_rng(w.rank)
    x = rng.normal(size=50)
    lme = dm.logmeanexp_over_ranks(dist, x)
    mx = dm.max_over_ranks(dist, float(w.rank))
    q.put((w.rank, sorted(allu), tot.tolist(), lme, mx))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    x = np.concatenate([np.random.default_rng(r).normal(size=50) for r in range(2)])
    want = np.log(np.mean(np.exp(x)))
    for rank, units, tot, lme, mx in res:
        assert units == list(range(10))
        assert tot == [55.0, 10.0]
        assert abs(lme - want) < 1e-12
        assert mx == 1.0


def _fake_vintage(thisT, yreal, seed):
    """Deterministic stand-in for one vintage's mcmcVAR (CPU): log-score draws and a
    forecast mean that depend only on (thisT, seed)."""
    rng = np.random.default_rng(seed)
    ls = rng.normal(-20.0, 3.0, size=(40, 2))
    return ls, ls - 0.5, ls / 2, ls / 3, np.full((3, 4), float(thisT))


def _govar_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    dist, w = pkg.distributed.init("gloo")
    data = np.arange(60 * 3, dtype=float).reshape(60, 3)
    res = pkg.samplers.goVAR_batch(data, np.arange(60.0), [40, 45, 50, 55, 58], 2, 12, 10, 40, 4,
                                   np.ones(3), [2], dist=dist, run_vintage=_fake_vintage)
    q.put((w.rank, res["fcstYmvlogscore"].tolist(), res["fcstYhat"][0, 0].tolist(),
           res["assignment"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_govar_batch():
    """goVAR_batch over 5 vintages on 2 gloo ranks: LPT sharding, per-vintage log mean exp
    of the log-score draws (goVARshadowrateBlockHybrid.m:437-447), one all-gather; every
    rank ends with the same, complete per-vintage table equal to the world-1 result."""
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    data = np.arange(60 * 3, dtype=float).reshape(60, 3)
    ref = pkg.samplers.goVAR_batch(data, np.arange(60.0), [40, 45, 50, 55, 58], 2, 12, 10, 40, 4,
                                   np.ones(3), [2], run_vintage=_fake_vintage)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_govar_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, ls, yh, assign in res:
        assert sorted(assign[0] + assign[1]) == list(range(5)) and assign[0] and assign[1]
        assert np.allclose(ls, ref["fcstYmvlogscore"], rtol=0, atol=1e-12)
        assert yh == [40.0, 45.0, 50.0, 55.0, 58.0]
    x = _fake_vintage(40, None, 1012023)[0]
    assert abs(ref["fcstYmvlogscore"][0] - np.log(np.mean(np.exp(x)))) < 1e-10


def test_lpt_cost_model_matches_device_calibration(pkg):
    """distributed.unit_cost against the device calibration it was fitted on
    (profiles/r04s_lpt_calibration.json: full-run seconds of 15 OOS vintages measured one chain
    alone, tools/calibrate_lpt.py): the coefficients are the fitted ones, the model reproduces
    the fit, and every measured vintage lies within the fit's stated residual."""
    import json
    from conftest import ROOT
    cal = json.loads((ROOT / "profiles" / "r04s_lpt_calibration.json").read_text())
    dm = pkg.distributed
    assert dm.LPT_COEF["a_per_T"] == cal["coef"]["a_per_T"]
    assert dm.LPT_COEF["e_per_cens_month"] == cal["coef"]["e_per_cens_month"]
    for row, fit in zip(cal["rows"], cal["fit_s"]):
        got = dm.unit_cost(row["T"], 241, 20, n_cens=row["n_cens"])
        assert abs(got - fit) <= 1e-9 * fit, (row, got, fit)
        assert abs(got - row["full_run_s"]) <= (cal["max_rel_residual"] + 1e-9) * row["full_run_s"], row
