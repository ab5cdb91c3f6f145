"""Generate the real-data MCSE fixtures (tests/golden/mcse_real_{linear,bh}.npz): posterior
moments from ONE long oracle chain on the reference's own data file fredblockMD20-2022-09.csv
at the 2022-08 jump-off (N = 20, p = 12, T = 750, K = 241), with Geweke numerical standard
errors as Diagnostics.m:134-300 computes them (oracle/ccmm_oracle_stats.momentg).

  linear  BASELINE configs[1]: mcmcVAR.m sweeps (oracle.linear_sweep, CTA in
          the weighted-SYRK form: the same posterior as CTA.m), reference initialisation
          (mcmcVAR.m:197-206), BURN burn-in + KEEP kept sweeps.
  bh      BASELINE configs[2] (C3): mcmcVARshadowrateBlockHybrid.m sweeps at ELB = 0.25 with the
          reference's ELB schedule (:433-466): the Gibbs sampler (gibbsdrawShadowrates, 101
          passes) for m < MCMCburnin / 2, then 1000 PS proposals, accept-first, Gibbs fallback.
          CTAsys in the SYRK form, ELB conditionals in the stable residual form.

Quantities (a subset, so that 4.5 combined standard errors is a sharp bar): the intercept
and own first-lag coefficient of every equation, the first-lag coefficient of FEDFUNDS in
every equation, the subdiagonal of A, the diagonal of PHI, sqrtht at three months; bh adds the
shadow rates of 24 censored cells spread over the window.  Used by tests/test_gpu_mcse_real.py.

Run: python tools/make_mcse_real_fixture.py linear|bh [--keep 2000] [--burn 1000]
(CPU; linear ~15 min, bh ~1-2 h single-threaded).

Several independent chains (the bh intercepts mix slowly: effective sample size ~30 per
2000 draws, so one chain's spectral NSE is itself noisy): run each with its own seed and
--part-out FILE (in parallel processes), then --merge FILE ... pools them: the mean of the
chain means, NSE = sqrt(sum NSE_i^2) / nchains, plus the between-chain standard error.  The
committed bh fixture pools seeds 20243 and 30001-30006 (their part files:
tests/golden/mcse_bh_parts/), the linear one seeds 20243 and 40001-40006
(tests/golden/mcse_linear_parts/)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np

from oracle import ccmm_oracle as oracle
from oracle.ccmm_oracle_stats import momentg

TSEL = (0, 374, 749)
NCELLS = 24


def selection(N, p, ncode):
    """Row/column indices into PAI (K x N) of the selected coefficients."""
    ff = list(ncode).index("FEDFUNDS")
    rows, cols = [], []
    for j in range(N):
        rows += [0, 1 + j, 1 + ff]       # intercept, own lag 1, FEDFUNDS lag 1
        cols += [j, j, j]
    return np.array(rows), np.array(cols)


def quantities(PAI, A, PHI, sqrtht, sel, shadow=None, cells=None):
    r, c = sel
    N = A.shape[0]
    q = [PAI[r, c], A[np.arange(1, N), np.arange(N - 1)], np.diag(PHI), sqrtht[list(TSEL), :].ravel(order="F")]
    if shadow is not None:
        q.append(shadow.ravel(order="F")[cells])
    return np.concatenate(q)


def censored_cells(sNaN):
    """NCELLS censored cells (column-major index into Ns x elbT) spread over the window."""
    idx = np.flatnonzero(sNaN.ravel(order="F"))
    return idx[np.linspace(0, idx.size - 1, NCELLS).round().astype(int)]


def merge(kind, files):
    """Pool independent chains (each file one chain's moments) into the fixture."""
    parts = [dict(np.load(f)) for f in files]
    K = len(parts)
    pm = np.array([q["pmean"] for q in parts])
    ns = np.array([q["nse3"] for q in parts])
    keep = int(parts[0]["keep"])
    burn = int(parts[0]["burn"])
    for q in parts:
        assert int(q["keep"]) == keep and int(q["burn"]) == burn
    extra = {}
    if kind == "bh":
        acc = sum(int(q["accept"]) for q in parts)
        nps = K * (burn + keep - (burn // 2))
        extra = dict(cells=parts[0]["cells"], accept=acc, accept_rate=acc / nps)
    out = ROOT / "tests" / "golden" / f"mcse_real_{kind}.npz"
    # the spread of the independent chain means is an estimate of the pooled mean's standard
    # error that does not lean on the spectral NSE (which underestimates the slowest directions,
    # ESS ~30 per chain for the bh intercepts)
    np.savez(out, pmean=pm.mean(axis=0), nse3=np.sqrt((ns ** 2).sum(axis=0)) / K, pmean_chains=pm,
             se_between=pm.std(axis=0, ddof=1) / np.sqrt(K),
             nse3_chains=ns, seeds=np.array([int(q["seed"]) for q in parts]), nchains=K, burn=burn, keep=keep,
             tsel=parts[0]["tsel"], sel_rows=parts[0]["sel_rows"], sel_cols=parts[0]["sel_cols"],
             nproposals=parts[0]["nproposals"], **extra)
    print("wrote", out, "chains", K, "spread of chain means / pooled NSE (max):",
          float(np.max(pm.std(axis=0, ddof=1) / np.sqrt(K) / (np.sqrt((ns ** 2).sum(axis=0)) / K))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["linear", "bh"])
    ap.add_argument("--burn", type=int, default=1000)
    ap.add_argument("--keep", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=20243)
    ap.add_argument("--nproposals", type=int, default=1000)
    ap.add_argument("--part-out", default=None, help="write this chain's moments here")
    ap.add_argument("--merge", nargs="+", default=None, help="pool chain files into the fixture")
    args = ap.parse_args()
    if args.merge:
        return merge(args.kind, args.merge)
    fred = oracle.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
    mpm = oracle.set_minnesota_mean(fred["ncode"])
    thisT = len(fred["ydates"])
    rng = np.random.default_rng(args.seed)
    sel = selection(20, 12, fred["ncode"])
    draws = []
    t0 = time.time()
    acc = 0
    cells = None
    if args.kind == "linear":
        su = oracle.var_setup(thisT, 12, 12, fred["data"], fred["ydates"], mpm, True)
        st = oracle.init_state(su)
        for m in range(args.burn + args.keep):
            st = oracle.linear_sweep(st, su, oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI), cta_form="syrk")
            if m >= args.burn:
                draws.append(quantities(st["PAI"], st["A"], st["PHI"], st["sqrtht"], sel))
            if m % 100 == 0:
                print(m, f"{time.time() - t0:.0f}s", flush=True)
    else:
        from oracle import ccmm_oracle_bh as bh
        ndxS, ndxO, _ = oracle.set_shadow_yields(fred["ncode"], 0.25)
        e0 = oracle.elb_t0(fred["data"], ndxS, 0.25, 12)
        bs = bh.bh_setup(thisT, 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
        cells = censored_cells(bs.sNaN)
        st = bh.bh_init_state(bs)
        ps_from = -(-args.burn // 2)                          # m >= MCMCburnin / 2 (1-based m)
        for m in range(args.burn + args.keep):
            use_ps = (m + 1) >= ps_from
            crn = bh.bh_draw_crn(rng, bs, args.nproposals if use_ps else 0)
            st = bh.bh_sweep(st, bs, crn, elb_impl="stable", use_ps=use_ps, cta_form="syrk")
            acc += bool(st.get("ps_accept", 0))
            if m >= args.burn:
                draws.append(quantities(st["PAI"], st["A"], st["PHI"], st["sqrtht"], sel,
                                        st["shadowrate"], cells))
            if m % 50 == 0:
                print(m, f"{time.time() - t0:.0f}s", "accepted", acc, flush=True)
    D = np.array(draws)
    mg = momentg(D)
    out = Path(args.part_out) if args.part_out else ROOT / "tests" / "golden" / f"mcse_real_{args.kind}.npz"
    extra = {} if cells is None else dict(cells=cells, accept=acc)
    np.savez(out, pmean=mg["pmean"], pstd=mg["pstd"], nse=mg["nse"], nse1=mg["nse1"], nse2=mg["nse2"],
             nse3=mg["nse3"], burn=args.burn, keep=args.keep, seed=args.seed, tsel=np.array(TSEL),
             sel_rows=sel[0], sel_cols=sel[1], nproposals=args.nproposals, **extra)
    print("wrote", out, "nvar", D.shape[1], "seconds", round(time.time() - t0),
          "min rne3", float(np.min(mg["rne3"])))


if __name__ == "__main__":
    main()
