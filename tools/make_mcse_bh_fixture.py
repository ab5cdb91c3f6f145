"""Generate tests/golden/mcse_bh_toy.npz: posterior moments of the block-hybrid shadow-rate
BVAR-SV (mcmcVARshadowrateBlockHybrid.m sweep with the acceptance-sampling ELB branch at
every sweep: 1000 PS proposals, Gibbs fallback) on the toy panel of
tests/test_gpu_ps._toy_bs((114, 120), valley=True) from ONE long oracle chain
(ccmm_oracle_bh.bh_sweep(use_ps=True), numpy RNG), with Geweke numerical standard errors
(oracle/ccmm_oracle_stats.momentg, Diagnostics.m:134-300).  Used by tests/test_gpu_mcse_bh.py.
Run: python tools/make_mcse_bh_fixture.py  (~3 min, CPU)."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np

from oracle import ccmm_oracle as oracle
from oracle import ccmm_oracle_bh as bh
from oracle.ccmm_oracle_stats import momentg

BURN, KEEP, SEED, NP = 400, 2000, 20242, 1000
TSEL = (0, 70, 140)


def toy():
    spec = importlib.util.spec_from_file_location("tps", ROOT / "tests" / "test_gpu_ps.py")
    t = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(t)
    return t._toy_bs(bh, (114, 120), valley=True)


def quantities(st, bs):
    """PAI (column-major), free A entries (row-wise), vech(PHI), sqrtht at three months and
    the shadow rates of the censored cells (column-major over Ns x elbT)."""
    N = bs.lin.N
    A = st["A"]
    afree = np.concatenate([A[i, :i] for i in range(1, N)])
    return np.concatenate([st["PAI"].ravel(order="F"), afree, oracle.vech_lower(st["PHI"]),
                           st["sqrtht"][list(TSEL), :].ravel(order="F"),
                           st["shadowrate"].ravel(order="F")[bs.sNaN.ravel(order="F")]])


def main():
    bs = toy()
    st = bh.bh_init_state(bs)
    rng = np.random.default_rng(SEED)
    draws, acc = [], 0
    for m in range(BURN + KEEP):
        st = bh.bh_sweep(st, bs, bh.bh_draw_crn(rng, bs, NP), elb_impl="stable", use_ps=True)
        acc += bool(st.get("ps_accept", 0))
        if m >= BURN:
            draws.append(quantities(st, bs))
    D = np.array(draws)
    mg = momentg(D)
    out = ROOT / "tests" / "golden" / "mcse_bh_toy.npz"
    np.savez(out, pmean=mg["pmean"], pstd=mg["pstd"], nse=mg["nse"], nse3=mg["nse3"], burn=BURN,
             keep=KEEP, seed=SEED, nproposals=NP, tsel=np.array(TSEL))
    print("wrote", out, "nvar", D.shape[1], "accept rate", acc / (BURN + KEEP))


if __name__ == "__main__":
    main()
