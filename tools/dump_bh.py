"""Debug helper: run one block-hybrid CRN sweep of the C3 configuration on the GPU
and save the device state for offline comparison with the oracle."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import __graft_entry__ as ge  # noqa: E402
from helpers import bh_crn_flat, random_state  # noqa: E402
from oracle import ccmm_oracle as O, ccmm_oracle_bh as BH  # noqa: E402

pkg = ge.load_package()
fred = O.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
ndxS, ndxO, _ = O.set_shadow_yields(fred["ncode"], 0.25)
mpm = O.set_minnesota_mean(fred["ncode"])
e0 = O.elb_t0(fred["data"], ndxS, 0.25, 12)
bs = BH.bh_setup(len(fred["ydates"]), 12, 12, fred["data"], fred["ydates"], ndxS, ndxO, mpm, 0.25, e0)
burn = int(sys.argv[1]) if len(sys.argv) > 1 else 100
bs.gibbsburn = burn
lin = bs.lin
st = random_state(O, lin, seed=60)
rng = np.random.default_rng(60)
crn = BH.bh_draw_crn(rng, bs)
ctx = pkg.Context(0)
ch = pkg.Chains(ctx, N=lin.N, p=lin.p, T=lin.T, B=1, crn=True, model=pkg.MODEL_BLOCKHYBRID,
                Ns=3, elbTmax=bs.elbT, elb_gibbsburn=burn, elb=0.25)
ch.set_data(0, lin.Y, lin.X, lin.iVdiag, lin.iVb, lin.sPHI, lin.Vol_0mean, lin.Vol_0vcvsqrt)
ch.set_elb_model(bs.ndxS, bs.actualrateBlock)
ch.set_elb_slot(0, bs.elbT0, bs.sNaN)
ch.set_state(*[st[k][..., None] for k in ("PAI", "A", "sqrtht", "h", "sqrtPHI")])
ch.sweep(1, crn=bh_crn_flat(BH, crn, bs)[:, None, None])
g = ch.get_state()
S = ch.get_shadowrate()
X, Y = ch.get_xy()
(ROOT / "gpurun_out").mkdir(exist_ok=True)
np.savez(ROOT / f"gpurun_out/bh_dump_{burn}.npz", S=S[..., 0], X=X[..., 0], Y=Y[..., 0],
         **{k: v[..., 0] for k, v in g.items()})
print("saved", burn)
