"""Developer tool: device gibbsdrawShadowratesB3 output of tests/test_gpu_gibbs_b3.py's case, saved for
offline comparison with numpy restatements.  Usage: b3_debug.py OUT.npz"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import __graft_entry__ as ge
from test_gpu_gibbs_b3 import _case
pkg = ge.load_package()
ctx = pkg.Context(0)
res = {}
for mv in (False, True):
    Y, STATE0, ndxS, sNaN, p, A, Bm, SVol, u = _case(5, month_varying=mv)
    for burn in (0, 100):
        got = ctx.gibbs_shadowrates_b3(Y[..., None], STATE0[:, None], ndxS, sNaN, p, A[..., None], Bm[..., None],
                                       SVol[..., None], 0.25, burnin=burn, u=u[:, :, :burn + 1, None],
                                       month_varying=mv)
        res[f"mv{int(mv)}_b{burn}"] = got[..., 0, 0]
np.savez(sys.argv[1], **res)
print("saved", list(res))
