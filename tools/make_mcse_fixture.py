"""Generate tests/golden/mcse_toy.npz: posterior moments of the linear BVAR-SV (mcmcVAR.m
sweep) on the toy design of tests/helpers.toy_setup(N=4, p=2, Tobs=122, seed=11) from ONE
long oracle chain (oracle.linear_sweep, numpy RNG, seed 20241), with Geweke numerical
standard errors as Diagnostics.m:134-300 computes them (oracle/ccmm_oracle_stats.momentg).
Used by tests/test_gpu_mcse.py.  Run: python tools/make_mcse_fixture.py  (~2 min, CPU)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np

from helpers import toy_setup
from oracle import ccmm_oracle as oracle
from oracle.ccmm_oracle_stats import momentg

BURN, KEEP, SEED = 500, 2000, 20241
TSEL = (0, 59, 119)


def quantities(st, N):
    """PAI (K x N, column-major), the free entries of A (row-wise below the diagonal),
    vech(PHI) (PHI_((tril(PHI_))~=0), mcmcVAR.m:290) and sqrtht at three months."""
    A = st["A"]
    afree = np.concatenate([A[i, :i] for i in range(1, N)])
    return np.concatenate([st["PAI"].ravel(order="F"), afree, oracle.vech_lower(st["PHI"]),
                           st["sqrtht"][list(TSEL), :].ravel(order="F")])


def main():
    su = toy_setup(oracle, N=4, p=2, Tobs=122, seed=11)
    st = oracle.init_state(su)
    rng = np.random.default_rng(SEED)
    draws = []
    for m in range(BURN + KEEP):
        st = oracle.linear_sweep(st, su, oracle.draw_crn(rng, su.N, su.K, su.T, su.dPHI), cta_form="syrk")
        if m >= BURN:
            draws.append(quantities(st, su.N))
    D = np.array(draws)
    mg = momentg(D)
    out = ROOT / "tests" / "golden" / "mcse_toy.npz"
    np.savez(out, pmean=mg["pmean"], pstd=mg["pstd"], nse=mg["nse"], nse1=mg["nse1"], nse2=mg["nse2"],
             nse3=mg["nse3"], burn=BURN, keep=KEEP, seed=SEED, tsel=np.array(TSEL))
    print("wrote", out, "nvar", D.shape[1], "max rne3", float(np.max(mg["rne3"])),
          "min rne3", float(np.min(mg["rne3"])))


if __name__ == "__main__":
    main()
