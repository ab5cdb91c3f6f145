"""Debug: k_fcst mean path vs the oracle on test_gpu_fcst case 0 (B = 1)."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as ge
from oracle import ccmm_oracle as O, ccmm_oracle_fcst as F
from fcst_cases import fcst_inputs
pkg = ge.load_package()
fred = O.load_fred_csv(ROOT / "tests/golden/data/fredblockMD20-2022-09.csv")
d = fcst_inputs(O, fred, B=1)
y = d["ys"][0]
ctx = pkg.Context(0)
fY, fYc, yhat, sc, st = ctx.fcst(d["PAI"], d["invA"], d["logSV0"], d["sqrtPHI"], d["Xj"], y,
                                 d["yields"], d["elb"], d["H"], d["Nd"], d["svz"], d["z"])
r = F.fcst_draw(d["PAI"][..., 0], d["invA"][..., 0], d["logSV0"][:, 0], d["sqrtPHI"][..., 0], d["Xj"][:, 0], y,
                d["yields"], d["elb"], d["svz"][..., 0], d["z"][..., 0])
np.set_printoptions(precision=5, linewidth=200)
print("yhat dev h0..3\n", yhat[:6, :4, 0]); print("yhat orc h0..3\n", r[2][:6, :4])
print("fY dev\n", fY[:6, :3, 0, 0]); print("fY orc\n", r[0][:6, :3, 0])
print("scores dev", sc[..., 0]); print("scores orc", r[3])
