#!/usr/bin/env python
"""Throughput benchmark: Gibbs sweeps/sec of the linear BVAR-SV (N=20, p=12,
T=750, K=241) over B chains per GPU (BASELINE.json configs[1]).

A "step" is one Gibbs sweep (CTA -> A -> SV -> PHI, mcmcVAR.m:211-274) of all
B chains resident on the GPU.  The data are the reference's own
fredblockMD20-2022-09.csv (committed fixture), jump-off 2022-08 (T=750);
chains start from the reference initialisation (mcmcVAR.m:197-206) and draw
from the on-device Philox stream.  Draw storage (post-burn-in form,
mcmcVAR.m:289-292) is inside the timed region.

Multi-GPU: one process per GPU (torch.distributed.run); every rank runs its
own B chains (the vintage/chain parfor shards with no data-path collective),
so scaling is weak; the only collectives are the timing barrier and the
max-reduction of the elapsed time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix (AMD spec)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec


def _progress(msg):
    """Progress on stderr (the one JSON result line stays alone on stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget per process of each CPU-oracle baseline line (rank 0, N=1 only)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="kernel option (ccmm_set_option) for every context of the run; repeatable")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-fcst", action="store_true", help="skip the predictive-density line")
    ap.add_argument("--bh-steps", type=int, default=3,
                    help="timed sweeps of the block-hybrid secondary lines (configs[2]); 0 = skip")
    ap.add_argument("--bh-warmup", type=int, default=1)
    ap.add_argument("--bh-chains", default="256,1024,4096",
                    help="chains per GPU of the block-hybrid lines (comma list)")
    ap.add_argument("--hy-steps", type=int, default=3,
                    help="timed sweeps of the hybrid-model lines (mcmcVARhybridGibbs, K = 277); 0 = skip")
    ap.add_argument("--hy-chains", default="256,1024", help="chains per GPU of the hybrid lines")
    ap.add_argument("--oos-steps", type=int, default=3,
                    help="timed kept sweeps (with forecasts) of the OOS line (configs[3]); 0 = skip")
    ap.add_argument("--oos-chains", default="1,8,32", help="chains per vintage of the OOS lines")
    ap.add_argument("--oos-full-draws", type=int, default=1000,
                    help="MCMCdraws of the measured full configs[3] run (burn-in = kept = this, C = 1, all 164 "
                         "vintages LPT-sharded over the ranks, end-of-run log-score all-gather) and of the "
                         "longest vintage alone (the per-rank floor); 0 = skip (projection only)")
    ap.add_argument("--s120-steps", type=int, default=2,
                    help="timed sweeps of the S120 stress line (configs[4], N=120); 0 = skip")
    ap.add_argument("--s120-warmup", type=int, default=1)
    ap.add_argument("--s120-chains", default="112",
                    help="chains per GPU of the S120 lines (112: ~245 GB of the 288 GB HBM for the 120 "
                         "factored 1472 x 1472 systems per chain; (chains, groups) = (96, 1) / (96, 3) / (112, 2) / "
                         "(112, 4) measured 98.7 / 101.8 / 103.9 / 105.1 sweeps/s standalone, profiles/r04u_s120_configs.json; inside "
                         "the full bench run (112, 4) fell to 89.4 while (112, 2) holds 104.3, profiles/r04z_*)")
    ap.add_argument("--s120-groups", type=int, default=2,
                    help="chain groups (HIP streams driven from host threads) of the S120 lines")
    ap.add_argument("--s120-only", action="store_true", help="run only the S120 lines (probe)")
    ap.add_argument("--girf-draws", type=int, default=256,
                    help="MCMC draws of the block-hybrid GIRF line (generateGIRF2blockhybrid, 1000 shock "
                         "paths x 120 horizons x 12 sims per draw); 0 = skip")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="parallel single-thread CPU baseline processes (0: min(16, cpus))")
    return ap.parse_args()


def launch_ranks(n):
    """`bench.py --gpus N` outside a torch.distributed launcher: start N rank processes
    (one per GPU, torch.distributed.run, rendezvous on 127.0.0.1) as CHILDREN of this
    process, which never touches the GPU, and exit with their status.  Rank 0 prints the
    JSON line."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    _progress(f"launching {n} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        _progress(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; reporting the launched world")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        torch.cuda.set_device(local)
        dist_.init_process_group("nccl")
        dist = dist_

    if args.s120_only:
        import __graft_entry__ as ge
        pkg = ge.load_package()
        ctx = pkg.Context(local)

        def barrier0():
            ctx.synchronize()
        for b in args.s120_chains.split(","):
            print(json.dumps(bench_s120(pkg, ctx, int(b), args, rank, barrier0, None)), flush=True)
        return

    cpu = None
    if world == 1 and not args.no_cpu:
        # before the GPU is initialised: the baseline runs in spawned single-thread processes
        _progress("cpu baseline")
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_workers)
        _progress("cpu baseline done")

    import __graft_entry__ as ge
    pkg = ge.load_package()
    d = pkg.model.importdata_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    thisT = len(d["ydates"])  # jump-off 2022-08 (doMCMClinear.m:27,94)
    m = pkg.model.build_var(thisT, p, 12, d["data"], d["ydates"], mpm, True)
    B = args.chains
    ctx = pkg.Context(local)
    for kv in args.opt:  # A/B runs of a kernel option: this context and the samplers' (ccmm_run_batch) one
        name, val = kv.split("=")
        ctx.set_option(name, int(val))
        pkg.samplers.context(local).set_option(name, int(val))
    cap = args.warmup + args.steps
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, store_capacity=cap,
                    seed=1012023 + 7919 * rank)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])

    def barrier():
        ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    _progress("main line")
    ch.sweep(args.warmup, store=True)
    barrier()
    if not args.no_profile:
        ch.profile(True)
    t0 = time.perf_counter()
    ch.sweep(args.steps, store=True)
    barrier()
    elapsed = time.perf_counter() - t0
    ktimes = ch.kernel_times() if not args.no_profile else {}
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    draws = ch.get_draws()
    assert np.all(np.isfinite(draws["PAI_all"])), "non-finite draws"
    ch.close()
    fc = bench_predictive(pkg, ctx, d, B) if (rank == 0 and not args.no_fcst) else None
    # secondary lines (configs[2], configs[3]) run on every rank: own barrier/max-reduction
    bh = None
    _progress("secondary lines")
    if args.bh_steps > 0:
        bh = [bench_block_hybrid(pkg, ctx, d, int(b), args, rank, barrier, dist)
              for b in args.bh_chains.split(",") if b.strip()]
    hy = None
    if args.hy_steps > 0:
        hy = [bench_hybrid(pkg, ctx, d, int(b), args, rank, barrier, dist)
              for b in args.hy_chains.split(",") if b.strip()]
    s120 = None
    if args.s120_steps > 0:
        s120 = [bench_s120(pkg, ctx, int(b), args, rank, barrier, dist)
                for b in args.s120_chains.split(",") if b.strip()]
    girf = None
    if args.girf_draws > 0:
        girf = bench_girf(pkg, ctx, d, args.girf_draws, rank, barrier, dist)
    oos = None
    if args.oos_steps > 0:
        oos = [bench_oos(pkg, ctx, d, int(c), args, rank, barrier, dist, floor=(i == 0))
               for i, c in enumerate(x for x in args.oos_chains.split(",") if x.strip())]

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    N, K, T = m.N, m.K, m.T
    value = world * B * args.steps / elapsed
    out = {
        "metric": "Gibbs sweeps/sec (chains x vintages) N=20 p=12",
        "value": round(value, 3),
        "unit": "sweeps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "fredblockMD20-2022-09.csv (reference data fixture), jump-off 2022-08, "
                "reference initialisation, Philox draws",
        "config": {"workload": "configs[1]: linear BVAR-SV (mcmcVAR) N=20 p=12 T=750 K=241, "
                               f"{B} chains per GPU, one sweep of all chains per step",
                   "chains_per_gpu": B, "N": N, "p": p, "T": T, "K": K,
                   "parallelism": f"chains sharded over {world} GPU(s), no data-path collective"},
    }
    if ktimes:
        # dominant kernel = largest accumulated device time
        dom = max(ktimes, key=lambda k: ktimes[k][0])
        per = {k: round(v[0] / max(v[1], 1), 4) for k, v in ktimes.items() if v[1]}
        if ktimes.get("k_gram_chol_lag", (0, 0))[1]:
            # lag-structured Gram + Cholesky (+ inverse): N*[T*K(K+1) + K^3/3] flop per chain
            # (the explicit inverse's K^3/3 is not counted)
            kname = "k_gram_chol_lag"
            flop = B * N * (T * K * (K + 1) + K ** 3 / 3)
        elif ktimes.get("k_gram_chol", (0, 0))[1]:
            # fused weighted SYRK + Cholesky: N*[T*K(K+1) + K^3/3] flop per chain
            kname = "k_gram_chol"
            flop = B * N * (T * K * (K + 1) + K ** 3 / 3)
        else:
            kname = "k_gram_big"  # multi-equation Gram (large-system path): T K (K+1) per system
            flop = B * N * T * K * (K + 1)
        kms = ktimes[kname][0] / max(ktimes[kname][1], 1)
        ach = flop / (kms * 1e-3) / 1e12
        pmc, pmc_src = load_pmc()
        traffic = pmc.get(kname, {}).get("hbm_bytes")
        out["roofline"] = {"kernel": kname, "bound": "mfma", "achieved": round(ach, 3),
                           "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4),
                           "traffic": None if traffic is None else int(traffic),
                           "traffic_source": pmc_src if traffic is not None else None,
                           "flop_per_launch": int(flop), "avg_launch_ms": round(kms, 4)}
        pk = pmc.get(kname, {})
        if "SQ_VALU_MFMA_BUSY_CYCLES" in pk:
            # counter evidence (separate rocprofv3 --pmc pass over this workload, tools/pmc_summary.py):
            # MFMA pipe busy fraction over the kernel and the F64 MFMA flop the hardware executed
            # (algorithmic flop above excludes the padded diagonal tiles and the inverse)
            out["roofline"]["counters"] = {
                "mfma_busy_frac": round(pk.get("mfma_busy_frac", 0.0), 4),
                "mfma_f64_flop_per_launch": int(pk.get("mfma_f64_flop", 0.0)),
                "SQ_VALU_MFMA_BUSY_CYCLES": int(pk["SQ_VALU_MFMA_BUSY_CYCLES"]),
                "SQ_INSTS_VALU_MFMA_MOPS_F64": int(pk.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)),
                "GRBM_GUI_ACTIVE": int(pk.get("GRBM_GUI_ACTIVE", 0)),
                "source": pmc_src}
        # streamed (HBM-roofline) kernels: SURVEY §8d's B_SV = 33 T N bytes per chain-sweep, the SV
        # block's external I/O, split by where it happens: k_sv_mix reads logy2 and the previous h and
        # writes the KSC indicator (8 + 8 + 1 = 17 T N); k_sv_part writes h and sqrtht (16 T N).  The
        # mixture observation / inverse variance the two hand over and the shocks eta are the
        # implementation's own traffic (another 32 T N), visible in "traffic" (PMC), not in "achieved".
        hb = {}
        for kn, nbytes in (("k_sv_part", B * 16 * T * N), ("k_sv_mix", B * 17 * T * N)):
            if ktimes.get(kn, (0, 0))[1]:
                ms = ktimes[kn][0] / ktimes[kn][1]
                gbs = nbytes / (ms * 1e-3) / 1e9
                hb[kn] = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": int(nbytes),
                          "traffic": (None if pmc.get(kn, {}).get("hbm_bytes") is None
                                      else int(pmc[kn]["hbm_bytes"]))}
        out["hbm_kernels"] = hb
        out["kernel_ms_per_sweep"] = per
        out["dominant_kernel"] = dom
    if bh is not None:
        out["block_hybrid"] = bh
    if oos is not None:
        out["oos"] = oos
    if s120 is not None:
        out["s120"] = s120
    if hy is not None:
        out["hybrid"] = hy
    if girf is not None:
        out["girf"] = girf
    if fc is not None:
        out["predictive"] = fc
    if cpu is not None:
        out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_predictive(pkg, ctx, d, B, H=48, Nd=10, steps=5):
    """Predictive density of every kept draw (mcmcVAR.m:298-381, logscoreGaussian.m,
    logscoreGaussianCensored.m) on a real vintage: jump-off 2022-07 (thisT = Tdata - 1), so
    yrealized(:,1) is the 2022-08 data row (goVARshadowrateBlockHybrid.m:267-283), B chains
    of the linear model, Nd = 10 draws x 48 horizons per kept draw.  Device-resident: the
    forecast block runs inside the chain set after each stored sweep (ccmm_chains_set_fcst);
    the rate is B / (k_fcst launch time, HIP events on the set's stream).  The block-level
    ccmm_fcst call (host buffers in and out) is timed beside it as the PCIe-inclusive rate.
    Not part of a sweep."""
    import time as _t
    _progress(f"bench_predictive {B}")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    thisT = len(d["ydates"]) - 1
    m = pkg.model.build_var(thisT, p, 12, d["data"], d["ydates"], mpm, True)
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    yields = np.zeros(m.N, bool)
    yields[ndxY] = True
    yreal = pkg.samplers.realized_values(d["data"], thisT, H, ndxS, 0.25)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, store_capacity=steps + 2, seed=424242)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_fcst(H, Nd, yields, keep_paths=False)
    ch.set_fcst_slot(0, yreal[:, 0])
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(3, store=False)
    ch.sweep(1, store=True)
    ch.get_fcst()
    ch.profile(True)
    ch.sweep(steps, store=True)
    ctx.synchronize()
    kt = ch.kernel_times()
    fc = ch.get_fcst()
    assert np.all(np.isfinite(fc["scores"][:, :, 0, :])), "non-finite log scores"
    kms = kt["k_fcst"][0] / kt["k_fcst"][1]
    # the block-level call on the last state (PCIe-inclusive)
    stt = ch.get_state()
    ch.close()
    Xj = np.repeat(m.Xjumpoff[:, None], B, axis=1)
    args = (stt["PAI"], stt["invA"], stt["h"][m.T - 1], stt["sqrtPHI"], Xj, yreal[:, 0], yields, 0.25, H, Nd)
    ctx.fcst(*args, seed=5, sweep=0)
    t0 = _t.perf_counter()
    for r in range(3):
        ctx.fcst(*args, seed=5, sweep=r + 1)
    ms_host = (_t.perf_counter() - t0) * 1e3 / 3
    return {"workload": f"predictive density: {B} chains (linear, jump-off 2022-07, realized 2022-08) x "
                        f"{Nd} draws x {H} horizons per kept draw, linear + censored paths, RB mean, "
                        "4 one-step log scores",
            "value": round(B / (kms * 1e-3), 1), "unit": "chain-draws/s (device-resident, k_fcst)",
            "k_fcst_ms": round(kms, 4), "launches": int(kt["k_fcst"][1]),
            "ccmm_fcst_ms_per_call_pcie": round(ms_host, 3),
            "ccmm_fcst_chain_draws_per_s_pcie": round(B / (ms_host * 1e-3), 1),
            "mean_logscore": round(float(np.mean(fc["scores"][:, :, 0, :])), 4)}


def _oos_timed(S, ctx, units, C, ids, steps, barrier, H, Nd, profile):
    """Time one OOS chain set through the reference's three ELB phases: Gibbs burn-in
    sweeps, PS burn-in sweeps, kept sweeps (PS + stored draw + predictive density).
    Returns (seconds per phase for `steps` sweeps, kernel times, PS stats, status)."""
    import time as _t
    ch, _, _ = S._bh_chain_set(ctx, units, C, seed=1012023, ids=ids, store_capacity=steps + 1,
                                gibbsburn=100, ELBbound=0.25, ndxYIELDS=_OOS_NDXY[0], fcstNhorizons=H, Nd=Nd)
    # the reference's ELB schedule (mcmcVARshadowrateBlockHybrid.m:433-466): Gibbs for
    # m < MCMCburnin/2, then 1000 PS proposals with the Gibbs draw as fallback
    ch.set_elb_ps(1000, 2 + steps)
    ch.sweep(1, store=True)                       # warm-up (also the forecast path)
    ch.get_fcst()
    ch.get_draws()

    def timed(store):
        barrier()
        t0 = _t.perf_counter()
        ch.sweep(steps, store=store)
        barrier()
        return _t.perf_counter() - t0

    el_gibbs = timed(False)                       # m = 2 .. steps + 1: Gibbs burn-in
    el_burn = timed(False)                        # PS burn-in
    if profile:
        ch.profile(True)
    el_kept = timed(True)                         # PS + stored draw + predictive density
    kt = ch.kernel_times() if profile else {}
    fc = ch.get_fcst()
    assert np.all(np.isfinite(fc["fYsum"])), "non-finite forecasts"
    ch.profile(False)
    ps = ch.get_ps()
    st = ch.get_status()
    B = ch.B
    ch.close()
    return (el_gibbs, el_burn, el_kept), kt, ps, st, B


_OOS_NDXY = [None]


def bench_oos(pkg, ctx, d, C, args, rank, barrier, dist, H=48, Nd=10, floor=False):
    """BASELINE.json configs[3] (goVARshadowrateBlockHybrid quasi-real-time OOS): all 164
    vintages (jump-offs after 2008-12: T = 587..750, elbT = 2..165) x C chains as ONE
    device-resident chain set per GPU (vintages sharded over ranks longest-processing-time
    first), ELB Gibbs (101 passes) every sweep.  Timed: kept sweeps, each storing the draw
    and simulating the predictive density on the device (10 draws x 48 horizons per kept
    draw and chain, mcmcVARshadowrateBlockHybrid.m:550-625) plus the one-step log scores;
    then plain (burn-in) sweeps.  value = units x sweeps / time summed over ranks (fixed
    total work: strong scaling).  The projected OOS wall time is 1000 burn-in + 1000 kept
    sweeps per unit at these rates.

    floor=True also times the longest vintage alone (1 chain, T = 750, elbT = 165): the
    per-sweep latency no number of GPUs can go below, because one rank always holds that
    unit.  The expected N-GPU wall time of the line is max(floor run, 1-GPU run / N)."""
    _progress(f"bench_oos C={C}")
    p = 12
    S = pkg.samplers
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    _OOS_NDXY[0] = ndxY
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    Tj = [int(t) for t in (np.flatnonzero(d["ydates"] > S.datenum(2008, 12, 1)) + 1)]
    world = dist.get_world_size() if dist is not None else 1
    N, K = d["data"].shape[1], d["data"].shape[1] * p + 1
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    startELB = e0 + 1 + p
    costs = [pkg.distributed.unit_cost(t - p, K, N, n_cens=pkg.distributed.censored_months(
        d["data"], ndxS, 0.25, startELB, t)) for t in Tj]
    mine = pkg.distributed.lpt_assign(costs, world)[rank]
    units = S._bh_units(d["data"], d["ydates"], [Tj[v] for v in mine], p, 12, ndxS, ndxO, mpm,
                        0.25, e0, True, H)
    ids = np.array([v * C + c for v in mine for c in range(C)], dtype=np.uint32)
    steps = args.oos_steps
    (el_gibbs, el_burn, el_kept), kt, ps, st, B = _oos_timed(S, ctx, units, C, ids, steps, barrier, H, Nd,
                                                              not args.no_profile)
    if dist is not None:
        import torch
        tt = torch.tensor([el_kept, el_burn, el_gibbs], dtype=torch.float64, device=f"cuda:{ctx.device}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_kept, el_burn, el_gibbs = (float(x) for x in tt.tolist())
    units_total = len(Tj) * C
    kept = units_total * steps / el_kept
    burn = units_total * steps / el_burn
    gibbs = units_total * steps / el_gibbs
    n_ps = 2 * steps * B
    acc = int(ps["countAccept"].sum() + ps["countAcceptBurnin"].sum())
    proj = 500 * units_total / gibbs + 500 * units_total / burn + 1000 * units_total / kept
    res = {"workload": f"configs[3]: goVARshadowrateBlockHybrid OOS, {len(Tj)} vintages x {C} "
                       f"chain(s) = {units_total} units (T = 587..750, elbT = 2..165), one "
                       f"device-resident chain set per GPU, vintages LPT-sharded over {world} "
                       f"GPU(s); ELB schedule as the reference: Gibbs for m < 500, then 1000 PS "
                       f"proposals with Gibbs fallback",
           "value": round(kept, 3), "unit": "sweeps/s (kept sweeps incl. predictive density)",
           "burnin_ps_sweeps_per_s": round(burn, 3), "burnin_gibbs_sweeps_per_s": round(gibbs, 3),
           "ms_per_kept_step": round(1e3 * el_kept / steps, 3),
           "ms_per_burnin_ps_step": round(1e3 * el_burn / steps, 3),
           "ms_per_burnin_gibbs_step": round(1e3 * el_gibbs / steps, 3), "steps": steps,
           "ps_accept_rate": round(acc / max(n_ps, 1), 4),
           "forecast": f"{Nd} draws x {H} horizons per kept draw and chain + 4 one-step scores",
           "projected_full_run_s": round(proj, 1),
           "flagged_units": int(np.count_nonzero(st)), "scaling": "strong"}
    if floor and rank == 0:
        # the longest vintage alone: the per-rank latency floor of any sharding
        last = len(Tj) - 1
        u1 = S._bh_units(d["data"], d["ydates"], [Tj[last]], p, 12, ndxS, ndxO, mpm, 0.25, e0, True, H)
        (fg, fb, fk), _, _, _, _ = _oos_timed(S, ctx, u1, 1, np.array([last * C], np.uint32), steps,
                                              lambda: ctx.synchronize(), H, Nd, False)
        floor_s = (500 * fg + 500 * fb + 1000 * fk) / steps
        res["per_rank_floor"] = {
            "unit": f"vintage thisT = {Tj[last]} (T = {Tj[last] - p}, elbT = {Tj[last] - p - e0}), 1 chain",
            "ms_per_gibbs_step": round(1e3 * fg / steps, 3), "ms_per_ps_step": round(1e3 * fb / steps, 3),
            "ms_per_kept_step": round(1e3 * fk / steps, 3), "full_run_s": round(floor_s, 1),
            "expected_full_run_s": {str(n): round(max(floor_s, proj * world / n), 1) for n in (1, 2, 4, 8)},
            "note": "expected N-GPU wall time = max(longest vintage alone, this line's 1-GPU time / N): "
                    "LPT puts the longest vintage on some rank, whose sweep cannot run faster than "
                    "that unit's own latency"}
    if floor and args.oos_full_draws > 0:
        res.update(oos_full_run(pkg, ctx, d, args.oos_full_draws, rank, barrier, dist, Tj, H, Nd, proj, world))
    if kt:
        res["kernel_ms_per_sweep"] = {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]}
    return res


def oos_full_run(pkg, ctx, d, draws, rank, barrier, dist, Tj, H, Nd, proj, world):
    """configs[3] measured end to end (goVARshadowrateBlockHybrid.m:126-517 with one chain per vintage, as
    the reference runs it): every vintage's `draws` burn-in + `draws` kept sweeps with the predictive
    density, vintages LPT-sharded over the ranks, each rank's vintage loop in the library
    (ccmm_run_batch, engine="native"), then the end-of-run exchange of the per-vintage log scores and
    summaries (all_gather_object over RCCL) inside the timed region; max over ranks.  Beside it the
    longest vintage (thisT = Tj[-1]) alone, the same full length on rank 0: the latency floor of any
    sharding."""
    import time as _t
    S = pkg.samplers
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    kw = dict(MCMCdraws=draws, fcstNdraws=Nd * draws, fcstNhorizons=H, ELBbound=0.25, nchains=1,
              engine="native", chunk=100)
    _progress(f"oos full run: {len(Tj)} vintages x {draws} + {draws} sweeps on {world} rank(s)")
    barrier()
    t0 = _t.perf_counter()
    r = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, dist=dist,
                                           device=ctx.device, **kw)
    barrier()
    el = _t.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{ctx.device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ls = np.asarray(r["fcstYmvlogscore"], float)
    out = {"measured_full_run_s": round(el, 2),
           "measured_full_run": {
               "workload": f"{len(Tj)} vintages x 1 chain x ({draws} burn-in + {draws} kept) sweeps, fcstNdraws = "
                           f"{Nd * draws}, {H} horizons, reference ELB schedule; ccmm_run_batch per rank + "
                           "end-of-run all-gather of the per-vintage log scores (timed)",
               "seconds": round(el, 2), "ranks": world,
               "sweeps_per_s": round(len(Tj) * 2 * draws / el, 1),
               "finite_logscores": int(np.isfinite(ls).sum()),
               "mean_logscore": round(float(np.nanmean(ls)), 5),
               "retries": r["stats"]["retries"]}}
    if rank == 0:
        _progress(f"oos floor: vintage thisT = {Tj[-1]} alone, {draws} + {draws} sweeps")
        t0 = _t.perf_counter()
        rf = S.goVARshadowrateBlockHybrid_batch(d["data"], d["ydates"], ndxS, ndxO, mpm, Tjumpoffs=[Tj[-1]],
                                                device=ctx.device, **kw)
        ctx.synchronize()
        fl = _t.perf_counter() - t0
        out["per_rank_floor_measured"] = {
            "unit": f"vintage thisT = {Tj[-1]} alone, 1 chain, {draws} + {draws} sweeps (full length, measured)",
            "seconds": round(fl, 2)}
        ls0 = float(rf["fcstYmvlogscore"][0])
        if np.isfinite(ls0):
            out["per_rank_floor_measured"]["logscore"] = round(ls0, 5)
        else:  # the last vintage: no realized month after its jump-off to score (NaN, as the reference's)
            out["per_rank_floor_measured"]["logscore"] = None
            out["per_rank_floor_measured"]["logscore_note"] = "no realized month after the last vintage (NaN)"
        out["expected_full_run_s_measured"] = {str(n): round(max(fl, el * world / n), 1) for n in (1, 2, 4, 8)}
    return out


def bench_girf(pkg, ctx, d, M, rank, barrier, dist, nsim=1000, H=120):
    """generateGIRF2blockhybrid.m:199-259 on the device (ccmm_girf): M kept draws (synthetic
    stable draws of the N = 20, p = 12 block-hybrid VAR), nsim = 1000 shock paths x 4
    antithetic sets x 3 scenarios x 120 horizons each.  value = MCMC draws per second (units
    shared over ranks: each rank simulates M draws).  MFMA work: 12 nsim H 2 N (K + Ny p + N)
    algorithmic flop per draw."""
    _progress(f"bench_girf {M}")
    import time as _t
    N, p = 20, 12
    ndxS, ndxO, ndxY = pkg.model.setShadowYields(d["ncode"], 0.25)
    yields = np.zeros(N, bool)
    yields[ndxY] = True
    K, Ny = 1 + N * p, int(yields.sum())
    rng = np.random.default_rng(17 + rank)
    PAI = np.zeros((K, N, M))
    PAI[0] = 0.1 * rng.standard_normal((N, M))
    for l in range(p):
        PAI[1 + l * N:1 + (l + 1) * N] = ((0.5 / (l + 1) ** 2) * np.eye(N))[..., None] + \
            0.01 * rng.standard_normal((N, N, M))
    invA = np.repeat(np.eye(N)[..., None], M, -1) + 0.1 * np.tril(np.ones((N, N)), -1)[..., None] * \
        rng.standard_normal((N, N, M))
    sqrtPHI = np.repeat((0.1 * np.eye(N))[..., None], M, -1)
    SV0 = 0.5 + rng.random((N, M))
    Xj = np.vstack([np.ones((1, M)), 0.5 + 0.3 * rng.standard_normal((N * p + Ny * p, M))])
    kw = dict(bh=True, actual=~yields, ndxYields=yields, elb=0.25, cumcode=d["cumcode"], np_=12)
    ctx.girf(PAI[..., :2], invA[..., :2], sqrtPHI[..., :2], SV0[:, :2], Xj[:, :2], H, 64, 0.11, **kw)
    barrier()
    t0 = _t.perf_counter()
    out = ctx.girf(PAI, invA, sqrtPHI, SV0, Xj, H, nsim, 0.11, **kw)
    barrier()
    el = _t.perf_counter() - t0
    assert np.all(np.isfinite(out)), "non-finite GIRF"
    world = dist.get_world_size() if dist is not None else 1
    flop = 12.0 * nsim * H * 2 * N * (K + Ny * p + N) * M
    flop_mfma = 12.0 * nsim * H * 2 * 16 * ((N + 15) // 16) * 4 * ((K + Ny * p + N + 3) // 4) * M
    return {"workload": f"generateGIRF2blockhybrid: {M} MCMC draws x {nsim} shock paths x 4 antithetic "
                        f"sets x 3 scenarios x {H} horizons (N = {N}, p = {p}, {Ny} yields), one call "
                        f"incl. host<->device copies", "value": round(world * M / el, 2),
            "unit": "MCMC draws/s", "seconds": round(el, 3), "draws": M,
            "fp64_mfma": {"achieved": round(flop / el / 1e12, 2), "executed": round(flop_mfma / el / 1e12, 2),
                          "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(flop / el / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                          "note": "achieved = algorithmic flop (unpadded N x states) / wall time; executed "
                                  "counts the padded 16 x 16 x 4 tiles"}}


def bench_block_hybrid(pkg, ctx, d, B, args, rank, barrier, dist):
    """Secondary line, BASELINE.json configs[2] (doMCMCshadowrateBlockHybrid, ELB = 0.25):
    B chains of the block-hybrid shadow-rate sweep (CTAsys -> A -> SV -> PHI -> ELB Gibbs
    with gibbsburn + 1 = 101 passes and inverse-CDF truncated normals -> X/Y rebuild,
    mcmcVARshadowrateBlockHybrid.m:332-520) at the 2022-08 jump-off: elbT = 165 months,
    109 censored months / 276 censored cells.  Same timing protocol as the main line."""
    _progress(f"bench_block_hybrid {locals().get('B', locals().get('C'))}")
    import time as _t
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    bm = pkg.model.build_bh(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, ndxO, mpm,
                            0.25, e0, True)
    m = bm.var
    Ns = len(bm.ndxS)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False,
                    store_capacity=args.bh_warmup + args.bh_steps, seed=1012023 + 7919 * rank + 1,
                    model=pkg.MODEL_BLOCKHYBRID, Ns=Ns, elbTmax=bm.elbT, elb_gibbsburn=100,
                    elb=0.25)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(bm.ndxS, bm.actual_block)
    ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(args.bh_warmup, store=True)
    barrier()
    if not args.no_profile:
        ch.profile(True)
    t0 = _t.perf_counter()
    ch.sweep(args.bh_steps, store=True)
    barrier()
    el = _t.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{ctx.device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    S = ch.get_shadowrate()
    assert np.all(np.isfinite(S)), "non-finite shadow rates"
    world = dist.get_world_size() if dist is not None else 1
    ncens = int(np.any(bm.sNaN, axis=0).sum())
    res = {"workload": "configs[2]: block-hybrid shadow-rate BVAR-SV (mcmcVARshadowrateBlockHybrid) "
                       f"N=20 p=12 T={m.T} ELB=0.25, Ns={Ns}, elbT={bm.elbT}, {ncens} censored "
                       f"months / {int(bm.sNaN.sum())} cells, ELB Gibbs (101 passes) every sweep, "
                       f"{B} chains per GPU",
           "value": round(world * B * args.bh_steps / el, 3), "unit": "sweeps/s",
           "ms_per_step": round(1e3 * el / args.bh_steps, 4), "steps": args.bh_steps,
           "warmup": args.bh_warmup}
    if not args.no_profile:
        kt = ch.kernel_times()
        res["kernel_ms_per_sweep"] = {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]}
        # k_elb_gibbs streams each censored month's conditional record (elb_cond_stride
        # minus the Ns x Ns Omega block: 228 doubles at Ns=3, p=12) once per pass and reads
        # and writes the chain's Ns x elbT shadow rates once (ccmm_elb.hip k_elb_gibbs)
        if kt.get("k_elb_gibbs", (0, 0))[1]:
            # the ELB passes are bound by VALU issue and the dependent month-to-month chain, not by HBM
            # (the month records stay in L2): report the VALU issue fraction from the newest committed
            # PMC summary of this line (tools/gpu/pmc_issue.sh: SQ_INSTS_VALU x 4 cycles per wave64
            # instruction over the chip's SIMD cycles; profiles/*pmc_issue*.json), beside the record bytes
            rec = Ns + Ns * (Ns - 1) + Ns + 2 * p * Ns * Ns
            nbytes = B * (101 * ncens * rec * 8 + 2 * 8 * Ns * bm.elbT)
            ms = kt["k_elb_gibbs"][0] / kt["k_elb_gibbs"][1]
            gbs = nbytes / (ms * 1e-3) / 1e9
            res["elb_gibbs"] = {"bound": "valu-issue + dependent latency", "avg_launch_ms": round(ms, 4),
                                "record_bytes_per_launch": int(nbytes), "record_GBs": round(gbs, 1),
                                "note": "101 sequential passes per chain, up to 8 in flight as a wavefront"}
            pmc, src = load_pmc("*pmc_issue*.json")
            for kn in ("k_elb_gibbs_wf", "k_elb_gibbs_oct", "k_elb_gibbs"):
                if pmc.get(kn, {}).get("valu_issue_frac") is not None:
                    res["elb_gibbs"].update(valu_issue_frac=round(pmc[kn]["valu_issue_frac"], 4),
                                            issue_kernel=kn, issue_source=src,
                                            issue_note="PMC pass over the B = 256 block-hybrid sweep "
                                                       "(tools/kernel_times_bh.py 256)")
                    break
    ch.close()
    return res


def bench_hybrid(pkg, ctx, d, B, args, rank, barrier, dist):
    """Secondary line: the hybrid shadow-rate model (mcmcVARhybridGibbs.m, X = [1, lags,
    Xffrlags]: K = 241 + Ns p = 277, KP = 320, the generic fused Gram + Cholesky path with
    the ELB step), fredblockMD20 at the 2022-08 jump-off, ELB 0.25.  Same timing protocol."""
    import time as _t
    _progress(f"bench_hybrid {B}")
    p = 12
    mpm = pkg.model.setMinnesotaMean(d["ncode"])
    ndxS, _, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    hm = pkg.model.build_hybrid(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, mpm, 0.25, e0, True)
    m = hm.var
    Ns = len(hm.ndxS)
    ch = pkg.Chains(ctx, N=m.N, p=p, T=m.T, B=B, crn=False, store_capacity=args.hy_steps + 1,
                    seed=1012023 + 7919 * rank + 3, model=pkg.MODEL_HYBRID, Ns=Ns, elbTmax=hm.elbT,
                    elb_gibbsburn=100, elb=0.25)
    ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
    ch.set_elb_model(hm.ndxS, None)
    ch.set_elb_slot(0, hm.elbT0, hm.sNaN)
    st = pkg.model.initial_state(m, B)
    ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
    ch.sweep(1, store=True)
    barrier()
    if not args.no_profile:
        ch.profile(True)
    t0 = _t.perf_counter()
    ch.sweep(args.hy_steps, store=True)
    barrier()
    el = _t.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{ctx.device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    assert np.all(np.isfinite(ch.get_shadowrate())), "non-finite shadow rates"
    world = dist.get_world_size() if dist is not None else 1
    res = {"workload": f"hybrid shadow-rate BVAR-SV (mcmcVARhybridGibbs) N=20 p=12 T={m.T} K={m.K}, "
                       f"Ns={Ns}, elbT={hm.elbT}, ELB Gibbs (101 passes) every sweep, {B} chains per GPU",
           "value": round(world * B * args.hy_steps / el, 3), "unit": "sweeps/s",
           "ms_per_step": round(1e3 * el / args.hy_steps, 4), "steps": args.hy_steps, "warmup": 1}
    if not args.no_profile:
        kt = ch.kernel_times()
        res["kernel_ms_per_sweep"] = {k: round(v[0] / v[1], 4) for k, v in kt.items() if v[1]}
        if kt.get("k_gram_chol", (0, 0))[1]:
            K = m.K
            fl = B * m.N * (m.T * K * (K + 1) + K ** 3 / 3)
            ms = kt["k_gram_chol"][0] / kt["k_gram_chol"][1]
            ach = fl / (ms * 1e-3) / 1e12
            res["fp64_mfma"] = {"kernel": "k_gram_chol", "achieved": round(ach, 3), "peak": FP64_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4),
                                "flop_per_launch": int(fl), "avg_launch_ms": round(ms, 4)}
    ch.close()
    return res


def _in_threads(fns):
    """Run callables concurrently on host threads (the libccmm calls release the GIL), so
    chain groups on separate HIP streams overlap on the device; re-raises the first error."""
    import threading
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]


def bench_s120(pkg, ctx, B, args, rank, barrier, dist, groups=None):
    """Stress line, BASELINE.json configs[4]: the block-hybrid shadow-rate
    sweep at N = 120, p = 12, T = 750 (K = 1441) on the synthetic S120 panel
    (ccmmshadowratevar-code_amd/synthetic.py: four shadow rates, two other yields, the last
    ~15 % of months at the ELB).  Every block runs on the large path: multi-equation
    FP64-MFMA Gram + blocked MFMA Cholesky + per-chain solve (ccmm_big.hip), the large-N
    A / SV / PHI blocks (ccmm_bign.hip), the ELB Gibbs step (101 passes).

    The B chains form G groups (chain sets) on G HIP streams (one context each), driven
    from G host threads: the per-chain sequential blocks (SV recursion, CTA solve, ELB Gibbs;
    one workgroup per chain) of one group overlap the MFMA Gram/Cholesky of another.  Same
    timing protocol as the main line (barrier, K timed sweeps of every group, max over ranks);
    the CTA kernels are priced against the FP64 MFMA peak from their per-launch times."""
    _progress(f"bench_s120 {locals().get('B', locals().get('C'))}")
    import time as _t
    G = groups or args.s120_groups
    if B % G:
        G = 1
    Bg = B // G
    p = 12
    d = pkg.synthetic.s120()
    mpm = np.ones(d["data"].shape[1])
    ndxS, ndxO, _ = pkg.model.setShadowYields(d["ncode"], 0.25)
    e0 = pkg.model.elbT0_of(d["data"], ndxS, 0.25, p)
    bm = pkg.model.build_bh(len(d["ydates"]), p, 12, d["data"], d["ydates"], ndxS, ndxO, mpm,
                            0.25, e0, True)
    m = bm.var
    Ns = len(bm.ndxS)
    ctxs = [ctx] + [pkg.Context(ctx.device) for _ in range(G - 1)]
    chs = []
    for g, cx in enumerate(ctxs):
        ch = pkg.Chains(cx, N=m.N, p=p, T=m.T, B=Bg, crn=False,
                        store_capacity=args.s120_warmup + args.s120_steps,
                        seed=1012023 + 7919 * rank + 2, model=pkg.MODEL_BLOCKHYBRID, Ns=Ns,
                        elbTmax=bm.elbT, elb_gibbsburn=100, elb=0.25)
        ch.set_rng_ids(np.arange(g * Bg, (g + 1) * Bg, dtype=np.uint32))
        if G > 1:
            ch.set_mfma_lock(1)
        ch.set_data(0, m.Y, m.X, m.iVdiag, m.iVb, m.sPHI, m.Vol_0mean, m.Vol_0vcvsqrt)
        ch.set_elb_model(bm.ndxS, bm.actual_block)
        ch.set_elb_slot(0, bm.elbT0, bm.sNaN)
        st = pkg.model.initial_state(m, Bg)
        ch.set_state(st["PAI"], st["A"], st["sqrtht"], st["h"], st["sqrtPHI"])
        chs.append(ch)
    _in_threads([lambda c=c: c.sweep(args.s120_warmup, store=True) for c in chs])
    for cx in ctxs:
        cx.synchronize()
    barrier()
    if not args.no_profile:
        for c in chs:
            c.profile(True)
    t0 = _t.perf_counter()
    _in_threads([lambda c=c: c.sweep(args.s120_steps, store=True) for c in chs])
    for cx in ctxs:
        cx.synchronize()
    barrier()
    el = _t.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{ctx.device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    flagged = 0
    for c in chs:
        assert np.all(np.isfinite(c.get_shadowrate())), "non-finite shadow rates"
        flagged += int(np.count_nonzero(c.get_status()))
    world = dist.get_world_size() if dist is not None else 1
    N, K, T = m.N, m.K, m.T
    ncens = int(np.any(bm.sNaN, axis=0).sum())
    res = {"workload": "configs[4]: S120 block-hybrid shadow-rate BVAR-SV, synthetic panel "
                       f"N={N} p={p} T={T} K={K}, Ns={Ns}, elbT={bm.elbT}, {ncens} censored months, "
                       f"ELB Gibbs (101 passes) every sweep, {B} chains per GPU in {G} stream group(s)",
           "value": round(world * B * args.s120_steps / el, 4), "unit": "sweeps/s",
           "ms_per_step": round(1e3 * el / args.s120_steps, 3), "steps": args.s120_steps,
           "warmup": args.s120_warmup, "chains": B, "groups": G, "chains_flagged": flagged}
    if not args.no_profile:
        kt = {}
        for c in chs:  # per-launch device times (events on each group's stream), all groups
            for k, v in c.kernel_times().items():
                a = kt.get(k, (0.0, 0))
                kt[k] = (a[0] + v[0], a[1] + v[1])
        res["kernel_ms_per_launch"] = {k: round(v[0] / v[1], 3) for k, v in kt.items() if v[1]}
        # CTA on FP64 MFMA: Gram T K (K+1) and Cholesky K^3 / 3 per equation,
        # per launch of one group (Bg chains)
        fg, fc = Bg * N * T * K * (K + 1), Bg * N * K ** 3 / 3
        mf = {}
        for kn, fl in (("k_gram_big", fg), ("k_chol_big", fc)):
            if kt.get(kn, (0, 0))[1]:
                ms = kt[kn][0] / kt[kn][1]
                mf[kn] = {"achieved": round(fl / (ms * 1e-3) / 1e12, 3), "peak": FP64_MFMA_PEAK_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(fl / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                          "flop_per_launch": int(fl), "avg_launch_ms": round(ms, 3)}
        ach = B * N * (T * K * (K + 1) + K ** 3 / 3) / (1e-3 * res["ms_per_step"]) / 1e12
        mf["whole_sweep"] = {"achieved": round(ach, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4),
                             "note": "CTA Gram + Cholesky flop of all chains over the whole sweep time"}
        if G > 1:
            mf["note"] = "groups overlap on the device: per-launch times include contention"
        res["fp64_mfma"] = mf
    for c in chs:
        c.close()
    return res


def load_pmc(pattern="*_pmc.json"):
    """Per-kernel counters from the newest committed rocprofv3 PMC summary (profiles/<pattern>, written
    by tools/pmc_summary.py from separate passes: FETCH_SIZE / WRITE_SIZE over this same bench command
    for HBM bytes; the issue counters for the ELB passes)."""
    import re

    def natural(pth):  # r01_v11 after r01_v9
        return [int(x) if x.isdigit() else x for x in re.split(r"(\d+)", pth.name)]

    files = sorted((ROOT / "profiles").glob(pattern), key=natural)
    if not files:
        return {}, None
    try:
        return json.loads(files[-1].read_text()), f"profiles/{files[-1].name}"
    except (OSError, ValueError):
        return {}, None


def _cpu_worker(kind, budget_s, seed, q):
    """One single-threaded oracle process (parfor worker): as many sweeps of one chain as
    fit in budget_s.  kind: linear-kron | linear-syrk | blockhybrid."""
    import sys as _s
    _s.path.insert(0, str(ROOT))
    from threadpoolctl import threadpool_limits

    from oracle import ccmm_oracle as O
    fred = O.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = O.set_minnesota_mean(fred["ncode"])
    rng = np.random.default_rng(seed)
    n = 0
    with threadpool_limits(1):
        if kind == "blockhybrid":
            from oracle import ccmm_oracle_bh as BH
            ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
            e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
            bs = BH.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO,
                             mpm, 0.25, e0)
            st = BH.bh_init_state(bs)
            step = lambda st: BH.bh_sweep(st, bs, BH.bh_draw_crn(rng, bs), elb_impl="qr")
        else:
            su = O.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
            st = O.init_state(su)
            form = kind.split("-")[1]
            step = lambda st: O.linear_sweep(st, su, O.draw_crn(rng, su.N, su.K, su.T, su.dPHI),
                                             cta_form=form)
        t0 = time.perf_counter()
        while True:
            st = step(st)
            n += 1
            el = time.perf_counter() - t0
            if el > budget_s:
                break
    q.put((n, el))


def _cpu_line(kind, budget_s, workers, sample):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_cpu_worker, args=(kind, budget_s, 1000 + w, q)) for w in range(workers)]
    for p_ in ps:
        p_.start()
    res = [q.get(timeout=budget_s * 20 + 300) for _ in ps]
    for p_ in ps:
        p_.join(timeout=60)
    value = sum(n / el for n, el in res)
    nsw = sum(n for n, _ in res)
    return {"value": round(value, 4), "unit": "sweeps/s", "cores": workers, "kind": "port",
            "scope": f"per-GPU share of the host: {workers} of its cores",
            "per_core": round(value / workers, 4),
            "sample": f"{nsw} sweeps: {workers} single-thread processes (parfor-style, one chain "
                      f"each) x ~{budget_s:.0f} s, {sample}"}


def _physical_cores():
    """Physical cores of the host (sockets x cores per socket from /proc/cpuinfo)."""
    phys = set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if ":" in line:
                    k, v = (x.strip() for x in line.split(":", 1))
                    cur[k] = v
                elif cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        return None
    phys.discard((None, None))
    return len(phys) or None


def _cpp_line(budget_s, workers, model="linear", form="kron"):
    """The compiled restatement (oracle/cpu_sweep.cpp), `workers` single-thread processes at once, one chain
    each (parfor), real data T = 750, the reference initialisation: model "linear" = the sweep of
    mcmcVAR.m:211-274 as written (kron-materialised CTA, explicit inverse); "blockhybrid" = the sweep of
    mcmcVARshadowrateBlockHybrid.m:332-520 as written (kron CTAsys, gibbsdrawShadowrates with the QR
    smoothing weights and 101 Gibbs passes, the X / Y rebuild).  OpenBLAS, one thread per process."""
    import sys as _s
    import tempfile
    _s.path.insert(0, str(ROOT))
    from oracle import ccmm_oracle as O
    from oracle import cpu_baseline as CB
    fred = O.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = O.set_minnesota_mean(fred["ncode"])
    with tempfile.TemporaryDirectory() as td:
        sp = Path(td) / "state.bin"
        if model == "blockhybrid":
            from oracle import ccmm_oracle_bh as BH
            ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
            e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
            bs = BH.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
            CB.write_state(sp, bs.lin, BH.bh_init_state(bs), bs)
            what = ("the block-hybrid sweep as written (CTAsys.m kron form, gibbsdrawShadowrates.m QR smoothing "
                    "weights by dgeqrf, 101 Gibbs passes, drawTruncNormal), ELB 0.25, elbT = 165")
        else:
            su = O.var_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], mpm, True)
            CB.write_state(sp, su, O.init_state(su))
            what = "the linear sweep as written (CTA.m kron form, explicit inverse)"
        if form == "syrk":
            what = what.replace("kron form", "algorithmic weighted-SYRK form").replace(
                "as written", "in the algorithmic form").replace(", explicit inverse", ", Cholesky + triangular solves")
        procs = [CB.bench_process(sp, budget_s, 1000 + w, form=form) for w in range(workers)]
        res = [CB.bench_result(p_, budget_s * 20 + 300) for p_ in procs]
    value = sum(n / el for n, el in res)
    nsw = sum(n for n, _ in res)
    return {"value": round(value, 4), "unit": "sweeps/s", "cores": workers, "kind": "port",
            "scope": f"per-GPU share of the host: {workers} of its cores",
            "per_core": round(value / workers, 4),
            "sample": f"{nsw} sweeps: {workers} single-thread processes (parfor-style, one chain each) x "
                      f"~{budget_s:.0f} s of oracle/cpu_sweep.cpp, {what}, in C++ on OpenBLAS "
                      f"{CB.blas_path().rsplit('/', 1)[-1]}"}


def _cpp_oos_line(budget_s, workers, nsample=4):
    """configs[3] on the host: the 164 single-chain vintage units of the OOS run
    (goVARshadowrateBlockHybrid.m:258-303, one chain per vintage, 1000 + 1000 sweeps) as the compiled
    block-hybrid restatement as written (oracle/cpu_sweep.cpp, kron CTAsys, QR gibbsdrawShadowrates with 101
    Gibbs passes every sweep).  Measured: the per-sweep time of `nsample` vintages spread over the jump-offs
    (T = 587..750, 2..109 censored months), `workers` processes at once; projected: the per-sweep cost
    a T + e n_cens fitted to them (non-negative least squares), 2000 sweeps per vintage, the 164 units
    LPT-packed on `workers` single-thread workers (parfor).  The PS branch and the forecasts of the
    reference schedule are not restated on the host (every sweep runs the Gibbs ELB step, no forecast
    block), so this is the CPU time of the sweeps only."""
    import sys as _s
    import tempfile
    _s.path.insert(0, str(ROOT))
    from scipy.optimize import nnls

    from oracle import ccmm_oracle as O
    from oracle import ccmm_oracle_bh as BH
    from oracle import cpu_baseline as CB
    fred = O.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = O.set_minnesota_mean(fred["ncode"])
    ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
    e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
    yd = np.asarray(fred["ydates"], float)
    dec2008 = 733743.0  # datenum(2008, 12, 1)
    Tj = [int(t) for t in (np.flatnonzero(yd > dec2008) + 1)]
    feats = []
    for thisT in Tj:  # (T, censored months) of every vintage
        bs = BH.bh_setup(thisT, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
        feats.append((bs.lin.T, int(np.count_nonzero(np.any(bs.sNaN, axis=0)))))
    pick = sorted({int(round(x)) for x in np.linspace(0, len(Tj) - 1, nsample)})
    per = max(1, workers // len(pick))
    costs = []
    with tempfile.TemporaryDirectory() as td:
        procs = []
        for q in pick:
            bs = BH.bh_setup(Tj[q], 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
            sp = Path(td) / f"state{q}.bin"
            CB.write_state(sp, bs.lin, BH.bh_init_state(bs), bs)
            procs.append([CB.bench_process(sp, budget_s, 2000 + 10 * q + w) for w in range(per)])
        for q, ps in zip(pick, procs):
            res = [CB.bench_result(p_, budget_s * 20 + 300) for p_ in ps]
            costs.append(sum(el for _, el in res) / sum(n for n, _ in res))
    F = np.array([feats[q] for q in pick], float)
    coef, _ = nnls(F, np.array(costs))
    unit = np.array(feats, float) @ coef * 2000.0  # seconds per vintage unit (2000 sweeps)
    loads = np.zeros(workers)
    for u in sorted(unit, reverse=True):  # LPT over the parfor workers
        loads[np.argmin(loads)] += u
    wall = float(loads.max())
    return {"value": round(len(Tj) * 2000 / wall, 4), "unit": "sweeps/s", "cores": workers, "kind": "port",
            "workload": f"configs[3]: {len(Tj)} vintages x 1 chain x 2000 sweeps (Gibbs ELB step every sweep)",
            "projected_full_run_s": round(wall, 1), "projected": True,
            "per_sweep_s_measured": {f"thisT={Tj[q]} (T={feats[q][0]}, n_cens={feats[q][1]})": round(c, 5)
                                     for q, c in zip(pick, costs)},
            "fit_s_per_sweep": {"per_month_of_data": float(coef[0]), "per_censored_month": float(coef[1])},
            "sample": f"{len(pick)} vintages x {per} single-thread processes x ~{budget_s:.0f} s of "
                      f"oracle/cpu_sweep.cpp (block-hybrid sweep as written), the rest projected by the fit; "
                      f"the 164 units LPT-packed on {workers} workers; no PS branch, no forecast block"}


def _cpp_s120_line(budget_s, workers):
    """configs[4] (S120: N = 120, p = 12, K = 1441, T = 750, Ns = 4) on the host: oracle/cpu_sweep.cpp's
    block-hybrid sweep with CTAsys in the algorithmic weighted-SYRK form (the kron form would materialise
    T (N - j + 1) x K = up to 1 GB per equation and ~11 TFLOP of CTA per sweep), `workers` processes of one
    chain each, at least one sweep each; gibbsdrawShadowrates as written (QR smoothing weights)."""
    import sys as _s
    import tempfile
    _s.path.insert(0, str(ROOT))
    from oracle import ccmm_oracle as O
    from oracle import ccmm_oracle_bh as BH
    from oracle import cpu_baseline as CB
    import __graft_entry__ as ge
    d = ge.load_package().synthetic.s120()
    ndxS, ndxO, _ = O.set_shadow_yields(d["ncode"], 0.25)
    e0 = O.elb_t0(d["data"], ndxS, 0.25, 12)
    bs = BH.bh_setup(len(d["ydates"]), 12, 12, d["data"], d["ydates"], ndxS, ndxO, np.ones(d["data"].shape[1]),
                     0.25, e0)
    with tempfile.TemporaryDirectory() as td:
        sp = Path(td) / "s120.bin"
        CB.write_state(sp, bs.lin, BH.bh_init_state(bs), bs)
        procs = [CB.bench_process(sp, budget_s, 3000 + w, form="syrk") for w in range(workers)]
        res = [CB.bench_result(p_, budget_s * 40 + 900) for p_ in procs]
    value = sum(n / el for n, el in res)
    nsw = sum(n for n, _ in res)
    return {"value": round(value, 5), "unit": "sweeps/s", "cores": workers, "kind": "port",
            "workload": "configs[4] S120 block hybrid, N = 120, K = 1441, T = 750, Ns = 4, elbT = 114",
            "s_per_sweep_per_process": round(sum(el for _, el in res) / nsw, 2),
            "sample": f"{nsw} sweeps: {workers} single-thread processes x >= 1 sweep of oracle/cpu_sweep.cpp "
                      f"(CTAsys in the weighted-SYRK form, gibbsdrawShadowrates as written), OpenBLAS"}


def cpu_baseline(budget_s, workers=0):
    """The reference algorithm restated on the host (oracle/; MATLAB cannot run here),
    parfor-style: `workers` single-thread processes, one chain each, real data T = 750.
    The reported ``cpu_baseline`` is the compiled C++ restatement of the linear sampler as written
    (oracle/cpu_sweep.cpp: kron-materialised X_j, explicit inverse, CTA.m:69-78; OpenBLAS); beside it
     the compiled block-hybrid sampler as written (kron CTAsys, the QR smoothing weights
    of gibbsdrawShadowrates.m:74-127, 101 Gibbs passes) and the numpy linear sweep in the SYRK form."""
    import os
    if workers <= 0:
        workers = min(16, os.cpu_count() or 1)   # the GPU box's CPU share for one GPU
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    blas = "unknown"
    try:
        from threadpoolctl import threadpool_info
        info = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        if info:
            blas = f"{info[0].get('internal_api')} {info[0].get('version')}"
    except Exception:
        pass
    env = f"numpy/scipy, BLAS {blas} (1 thread per process), CPU {cpu}, {os.cpu_count()} " \
          f"logical CPUs visible"
    lin = _cpp_line(budget_s, workers)
    lin["sample"] += f", CPU {cpu}"
    ncore = _physical_cores()
    # the whole host: a GPU job on the box is allotted 16 of its CPUs, so the
    # whole-host figure is the measured per-core rate x the physical cores; the per-core rate is also
    # measured with ONE process (no neighbour on the memory system) to show the 16-process rate holds
    one = _cpp_line(max(2.0, budget_s / 3), 1)
    if ncore:
        lin["all_host_cores"] = {
            "value": round(lin["per_core"] * ncore, 3), "unit": "sweeps/s", "cores": ncore,
            "kind": "port", "cpu": cpu, "blas": blas, "projected": True,
            "per_core_1_process": one["per_core"], f"per_core_{workers}_processes": lin["per_core"],
            "method": f"projected: measured per-core rate of the {workers}-process line x {ncore} physical "
                      f"cores (one single-thread parfor worker per core; the box allots a GPU job {workers} "
                      f"CPUs, so more processes are not run; 1-process per-core rate {one['per_core']})"}
    bh = _cpp_line(budget_s, workers, model="blockhybrid")
    bh["sample"] += f", CPU {cpu}"
    if ncore:
        bh["all_host_cores"] = {"value": round(bh["per_core"] * ncore, 3), "unit": "sweeps/s", "cores": ncore,
                                "projected": True, "method": "measured per-core rate x physical cores"}
    bh_syrk = _cpp_line(budget_s, workers, model="blockhybrid", form="syrk")
    bh_syrk["sample"] += f", CPU {cpu}"
    lin["lines"] = {
        "blockhybrid_cpp": bh,
        "blockhybrid_cpp_syrk": bh_syrk,
        "oos_configs3_cpp": _cpp_oos_line(max(3.0, budget_s / 2), workers),
        "s120_cpp_syrk": _cpp_s120_line(1.0, workers),
        "linear_numpy": _cpu_line("linear-syrk", max(2.0, budget_s / 3), workers,
                                  "linear sweep, algorithmic CTA (weighted SYRK + Cholesky + "
                                  "triangular solves) in numpy, " + env),
    }
    return lin


if __name__ == "__main__":
    main()
