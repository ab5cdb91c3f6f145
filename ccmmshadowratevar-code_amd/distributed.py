"""Multi-GPU layout of the quasi-real-time batch (goVARshadowrateBlockHybrid.m:258).

The reference runs ``parfor ndxT = 1:Njumpoffs`` with one chain per vintage and
no communication during sampling.  Here every (vintage, chain) unit is
independent for all sweeps, so units are sharded over ranks (one process per
GPU, torch.distributed over RCCL) with no data-path collective:

  * all chains of a vintage stay on one rank (quantiles, CRPS and log scores of
    that vintage need no cross-rank data, goVARshadowrateBlockHybrid.m:331-456);
  * vintages are assigned longest-processing-time first with the per-chain
    sweep cost model of SURVEY.md §8e (CTA grows with T, the ELB step with the
    censored months of the vintage);
  * the only collectives run at the end of the run: an all-gather of the
    per-vintage summaries and an all-reduce of global moments, plus the
    timing barrier/max of the benchmark.
"""
from __future__ import annotations

import heapq
import os
from dataclasses import dataclass

import numpy as np


@dataclass
class World:
    rank: int
    size: int
    local_rank: int


def world_from_env() -> World:
    return World(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                 int(os.environ.get("LOCAL_RANK", "0")))


# Measured per-vintage cost of the OOS run (tools/calibrate_lpt.py on one MI355X, one chain per vintage
# alone, 500 Gibbs + 500 PS + 1000 kept sweeps; profiles/r04s_lpt_calibration.json): seconds of a full
# run = a T + e n_cens at N = 20, K = 241 (NNLS fit over 15 vintages, max relative residual 0.14; the
# wavefront-step term of the fit came out zero: the ELB passes scale with the censored months).
LPT_COEF = {"a_per_T": 0.017482263240311456, "e_per_cens_month": 0.06402049319623504}


def unit_cost(T, K, N, n_cens=0, Nstate=None, Ny=None, passes=101, coef=None):
    """Per-chain cost of one vintage for the LPT assignment, calibrated on the device:
    the measured per-T term (CTA, SV, A-step: per-chain latency kernels, scaled by the CTA work
    N K^2 relative to the calibration system) plus the measured per-censored-month term of the
    ELB step (scaled by the passes and the state size relative to the calibration)."""
    c = LPT_COEF if coef is None else coef
    scale_t = (N * K * K) / (20.0 * 241.0 * 241.0)
    f = c["a_per_T"] * T * scale_t
    if n_cens:
        Nstate = N * 12 if Nstate is None else Nstate
        Ny = N if Ny is None else Ny
        f += c["e_per_cens_month"] * n_cens * (passes / 101.0) * ((Nstate + Ny) / 260.0)
    return float(f)


def elb_wavefront_steps(n_cens, passes=101, p=12, waves=8):
    """Serial steps of the ELB Gibbs passes of one chain (gibbsdrawShadowrates.m:181-245 as the
    device runs them, k_elb_gibbs_wf): pass n may draw censored month i once pass n - 1 is p months
    past it, so min(waves, n_cens / (p + 1)) passes are in flight (at least one)."""
    if n_cens <= 0:
        return 0.0
    weff = min(float(waves), max(1.0, n_cens / (p + 1.0)))
    return passes * n_cens / weff + (n_cens if weff > 1.0 else 0.0)


def censored_months(data, ndxS, elb, startELB, thisT):
    """Censored months of one vintage: rows startELB..thisT (1-based, the vintage's ELB
    window, goVARshadowrateBlockHybrid.m:131-134) in which some shadow-rate series sits at
    or below the ELB (mcmcVARshadowrateBlockHybrid.m:163-171).  The ELB Gibbs passes cost
    one conditional draw per censored cell, so this (not the window length) drives the
    vintage's ELB cost; after the 2015 lift-off the window grows while it does not."""
    d = np.asarray(data, float)[:, np.asarray(ndxS, int)]
    lo, hi = max(int(startELB) - 1, 0), int(thisT)
    if hi <= lo:
        return 0
    return int(np.count_nonzero(np.any(d[lo:hi] <= elb, axis=1)))


def lpt_assign(costs, world_size):
    """Longest-processing-time-first assignment of units to ranks.
    Returns a list (per rank) of unit indices, each sorted ascending."""
    costs = np.asarray(costs, float)
    order = np.argsort(-costs, kind="stable")
    heap = [(0.0, r) for r in range(world_size)]
    heapq.heapify(heap)
    out = [[] for _ in range(world_size)]
    for u in order:
        load, r = heapq.heappop(heap)
        out[r].append(int(u))
        heapq.heappush(heap, (load + costs[u], r))
    return [sorted(x) for x in out]


def shard_range(n, world_size, rank):
    """Contiguous block of n equal-cost units for `rank` (chains of one vintage)."""
    base, rem = divmod(n, world_size)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def init(backend=None, min_world=2):
    """Initialise torch.distributed from the torchrun environment (RCCL on GPU,
    gloo on CPU).  Returns (dist module or None, World); None below min_world ranks
    (min_world=1 forms a one-rank group, which runs the collectives' code paths)."""
    w = world_from_env()
    if w.size < min_world:
        return None, w
    import torch
    import torch.distributed as dist
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(w.local_rank)
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return dist, w


def _device_for(dist):
    import torch
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(dist, arr):
    """Global sum of per-rank moment arrays (posterior means / second moments)."""
    a = np.asarray(arr, np.float64)
    if dist is None:
        return a.copy()
    import torch
    t = torch.as_tensor(a.copy(), device=_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def logmeanexp_over_ranks(dist, local_logs):
    """log(mean(exp(x))) over the union of every rank's draws (log scores,
    goVARshadowrateBlockHybrid.m:437-447): allreduce-MAX then allreduce-SUM."""
    x = np.asarray(local_logs, np.float64).ravel()
    m = max_over_ranks(dist, x.max() if x.size else -np.inf)
    s = allreduce_sum(dist, np.array([np.exp(x - m).sum(), float(x.size)]))
    return float(m + np.log(s[0] / s[1]))


def gather_summaries(dist, local: dict, units_per_rank):
    """All-gather per-unit summary arrays (same shape per unit) into unit order.
    local maps unit index -> array."""
    keys = sorted(local)
    if dist is None:
        return {k: np.asarray(local[k]) for k in keys}
    objs = [None] * dist.get_world_size()
    dist.all_gather_object(objs, {k: np.asarray(v) for k, v in local.items()})
    out = {}
    for d in objs:
        out.update(d)
    return dict(sorted(out.items()))
