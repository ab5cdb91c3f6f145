"""Probe: the large CTA block at the S120 shape (N = 120, p = 12, K = 1441, T = 750) through
the block-level C ABI (ccmm_cta), B chains, smooth-volatility states.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel times."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np

import __graft_entry__ as g

pkg = g.load_package()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
d = pkg.synthetic.s120()
mpm = np.ones(d["data"].shape[1])
m = pkg.model.build_var(len(d["ydates"]), 12, 12, d["data"], d["ydates"], mpm, True)
rng = np.random.default_rng(0)
N, K, T = m.N, m.K, m.T
st = pkg.model.initial_state(m, 1)
A = np.repeat((np.eye(N) + np.tril(rng.uniform(-0.1, 0.1, (N, N)), -1))[..., None], B, axis=2)
h = np.cumsum(0.03 * rng.standard_normal((T, N, B)), axis=0) + np.log(np.var(m.Y, axis=0))[None, :, None]
sq = np.exp(h / 2)
PAI = np.repeat(st["PAI"], B, axis=2)
z = rng.standard_normal((K, N, B))
ctx = pkg.Context(0)
for r in range(reps):
    t0 = time.perf_counter()
    out, status = ctx.cta(m.Y, m.X, A, sq, m.iVdiag, m.iVb, PAI, z)
    el = time.perf_counter() - t0
    print(f"rep {r}: {el * 1e3:.1f} ms (incl. uploads), status {status.any()}, finite {np.isfinite(out).all()}",
          flush=True)
flop_gram = B * N * T * K * (K + 1)
flop_chol = B * N * K ** 3 / 3
print(f"B={B}: Gram {flop_gram / 1e9:.1f} GFLOP, Cholesky {flop_chol / 1e9:.1f} GFLOP per call")
