"""Generate the OOS-vintage posterior fixture (tests/golden/mcse_oos_vintage.npz): the predictive
density of ONE quasi-real-time vintage of goVARshadowrateBlockHybrid.m (block-hybrid model at ELB
0.25, the reference's ELB schedule: Gibbs for m < MCMCburnin / 2, then 1000 PS proposals with the
Gibbs fallback) from long oracle chains, with Geweke NSEs (Diagnostics.m:134-300, 15 % taper).

Per kept sweep the chain simulates fcstNdraws / MCMCdraws = 10 forecast paths over 48 horizons
(mcmcVARshadowrateBlockHybrid.m:550-625, oracle/ccmm_oracle_fcst.fcst_draw_bh) and records
  dens   mean over the 10 draws of exp(fcstLogscoreDraws) (the one-step predictive density at the
         realised values; goVARshadowrateBlockHybrid.m:437-439 takes log mean exp over all draws, so
         fcstYmvlogscore = log of the posterior mean of dens)
  lsc    mean over the 10 draws of fcstLogscoreDraws (a lighter-tailed companion of dens)
  paths  the mean of the censored paths (fcstYdraws: yields floored at the ELB, :696-700) at
         horizons 1, 12, 24, 48 for every variable (fcstYhat, :450)
Used by tests/test_gpu_mcse_oos.py.  CPU: CTAsys in the SYRK form, ELB conditionals in the stable
residual form, about 10 min per chain at the default vintage.

Run several chains in parallel (--seed S --part-out FILE), then --merge FILE ... pools them (the mean of
the chain means, NSE = sqrt(sum NSE_i^2) / nchains, plus the between-chain standard error)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np

from oracle import ccmm_oracle as oracle
from oracle import ccmm_oracle_bh as bh
from oracle import ccmm_oracle_fcst as F
from oracle.ccmm_oracle_stats import momentg

VINTAGE = 12          # index into Tjumpoffs (goVARshadowrateBlockHybrid.m:127): 2009-12
HSEL = (0, 11, 23, 47)
H, ND, ELB = 48, 10, 0.25


def vintage_thisT(ydates):
    from datetime import date
    dn = date(2008, 12, 1).toordinal() + 366
    Tj = np.flatnonzero(np.asarray(ydates) > dn) + 1
    return int(Tj[VINTAGE])


def yrealized(data, thisT, ndxS):
    """goVARshadowrateBlockHybrid.m:267-283."""
    Tdata, N = data.shape
    yr = np.full((N, H), np.nan)
    n = max(0, min(H, Tdata - thisT))
    yr[:, :n] = data[thisT:thisT + n].T
    ys = yr[ndxS, :]
    ys[ys < ELB] = ELB
    yr[ndxS, :] = ys
    return yr


def merge(files):
    parts = [dict(np.load(f)) for f in files]
    K = len(parts)
    pm = np.array([q["pmean"] for q in parts])
    ns = np.array([q["nse3"] for q in parts])
    out = ROOT / "tests" / "golden" / "mcse_oos_vintage.npz"
    np.savez(out, pmean=pm.mean(axis=0), nse3=np.sqrt((ns ** 2).sum(axis=0)) / K, pmean_chains=pm,
             se_between=pm.std(axis=0, ddof=1) / np.sqrt(K), seeds=np.array([int(q["seed"]) for q in parts]),
             nchains=K, burn=int(parts[0]["burn"]), keep=int(parts[0]["keep"]), thisT=int(parts[0]["thisT"]),
             hsel=parts[0]["hsel"], nproposals=int(parts[0]["nproposals"]),
             accept=sum(int(q["accept"]) for q in parts))
    print("wrote", out, "chains", K)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--burn", type=int, default=1000)
    ap.add_argument("--keep", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=50001)
    ap.add_argument("--nproposals", type=int, default=1000)
    ap.add_argument("--part-out", default=None)
    ap.add_argument("--merge", nargs="+", default=None)
    args = ap.parse_args()
    if args.merge:
        return merge(args.merge)
    from threadpoolctl import threadpool_limits
    fred = oracle.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    thisT = vintage_thisT(fred["ydates"])
    ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], ELB)
    ndxY = np.union1d(ndxS, ndxO)
    yields = np.zeros(fred["data"].shape[1], bool)
    yields[ndxY] = True
    e0 = oracle.elb_t0(fred["data"], ndxS, ELB, 12)
    bs = bh.bh_setup(thisT, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, ELB, e0)
    yr = yrealized(fred["data"], thisT, ndxS)
    data_v = fred["data"][:thisT]
    N, p = bs.lin.N, 12
    rng = np.random.default_rng(args.seed)
    st = bh.bh_init_state(bs)
    ps_from = -(-args.burn // 2)                              # m >= MCMCburnin / 2 (:435)
    acc = 0
    rows = []
    t0 = time.time()
    with threadpool_limits(1):
        for m in range(args.burn + args.keep):
            use_ps = (m + 1) >= ps_from
            crn = bh.bh_draw_crn(rng, bs, args.nproposals if use_ps else 0)
            st = bh.bh_sweep(st, bs, crn, elb_impl="stable", use_ps=use_ps, cta_form="syrk")
            acc += bool(st.get("ps_accept", 0))
            if m >= args.burn:
                Xj = F.bh_jumpoff(st["Y"], data_v, p, yields)
                svz = rng.standard_normal((N, H * ND))
                z = rng.standard_normal((N, H, ND))
                fY, sc = F.fcst_draw_bh(st["PAI"], st["invA"], st["h"][-1], st["sqrtPHI"], Xj, yr[:, 0], yields,
                                        bs.actualrateBlock, ELB, svz, z)
                fYc = fY.copy()
                fYc[yields] = np.maximum(fYc[yields], ELB)
                dens = np.mean(np.exp(sc[0]))
                rows.append(np.concatenate([[dens, np.mean(sc[0])], fYc.mean(axis=2)[:, list(HSEL)].ravel(order="F")]))
            if m % 100 == 0:
                print(m, f"{time.time() - t0:.0f}s", flush=True)
    D = np.array(rows)
    g = momentg(D)
    res = dict(pmean=g["pmean"], nse3=g["nse3"], seed=args.seed, burn=args.burn, keep=args.keep, thisT=thisT,
               hsel=np.array(HSEL), nproposals=args.nproposals, accept=acc)
    out = args.part_out or str(ROOT / "tests" / "golden" / "mcse_oos_vintage.npz")
    np.savez(out, **res)
    print("wrote", out, f"thisT {thisT} elbT {bs.elbT}, {time.time() - t0:.0f}s, PS accepts {acc}")


if __name__ == "__main__":
    main()
